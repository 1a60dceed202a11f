"""Frame RMS kernels (GPU) against a sequential float32 fold in numpy: bit-exact.

The reference's frame RMS (silence.rs:154-169 for trimming, energy_flux.rs:122-131 for the
energy-flux onsets) is sqrt(sum_k (x_k g)^2 / len) with the sum folded in sample order.  The
engine's default kernel (k_frame_rms_run) streams each run of 4G frames once (G = frame / hop)
with G accumulators in flight; the per-frame kernel (k_frame_rms) serves other hops.  Cases:
every G the stream kernel takes (1, 2, 4, 8), a hop it does not (441), tracks shorter than a
frame, tracks of exactly one frame, odd lengths and offsets (unaligned 16-B blocks), runs that
cross track boundaries, and the per-frame kernel on the same inputs.
"""
import numpy as np
import pytest

import sdsp

pytestmark = pytest.mark.gpu

LENS = [100, 2048, 2049, 5000, 44100 * 3 + 7, 1, 3071, 44100 + 513, 0, 9001, 2 * 44100 + 3]


def _ref(tracks, gains, fs, hop):
    out = []
    for x, g in zip(tracks, gains):
        n = x.size
        if n == 0:
            continue
        nf = (n - fs) // hop + 1 if n >= fs else 1
        y = (x * np.float32(g)).astype(np.float32)
        yy = (y * y).astype(np.float32)
        for f in range(nf):
            s = f * hop
            e = min(s + fs, n)
            seg = yy[s:e]
            tot = np.cumsum(seg, dtype=np.float32)[-1] if seg.size else np.float32(0.0)
            out.append(np.sqrt(np.float32(tot) / np.float32(e - s)) if e > s else np.float32(0.0))
    return np.array(out, np.float32)


def _tracks(seed):
    rng = np.random.default_rng(seed)
    xs = [(rng.standard_normal(n) * 0.3).astype(np.float32) for n in LENS]
    xs[4][1000:30000] = 0.0  # digital silence inside a track
    gains = rng.uniform(0.5, 2.0, len(xs)).astype(np.float32)
    return xs, gains


@pytest.mark.parametrize("fs,hop", [(2048, 512), (2048, 1024), (1024, 1024), (4096, 512), (2048, 256), (2048, 441),
                                    (512, 128)])
def test_frame_rms_bit_exact(fs, hop):
    xs, gains = _tracks(fs + hop)
    ref = _ref(xs, gains, fs, hop)
    got = sdsp.debug_frame_rms(xs, gains, fs, hop)
    assert got.shape == ref.shape
    bad = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert bad == 0, f"{bad} of {ref.size} frames differ (max diff {np.max(np.abs(got - ref))})"
    per_frame = sdsp.debug_frame_rms(xs, gains, fs, hop, per_frame=True)
    assert np.array_equal(per_frame.view(np.uint32), got.view(np.uint32))


def test_frame_rms_many_tracks_ragged():
    """Hundreds of short ragged tracks: most 16-frame runs cross a track boundary."""
    rng = np.random.default_rng(5)
    xs = [(rng.standard_normal(int(n)) * 0.2).astype(np.float32) for n in rng.integers(1500, 12000, 300)]
    gains = rng.uniform(0.5, 2.0, len(xs)).astype(np.float32)
    for fs, hop in [(2048, 512), (2048, 1024)]:
        ref = _ref(xs, gains, fs, hop)
        got = sdsp.debug_frame_rms(xs, gains, fs, hop)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (fs, hop)
