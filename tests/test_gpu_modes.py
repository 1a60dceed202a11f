"""Engine modes and switches that must not change results (GPU, through the C ABI).

* SDSP_STAGES_BPM_ONLY (BASELINE config 5's "BPM-only" path: src/lib.rs:86-910, SURVEY rows
  a1-a19) gives a full run's bpm, bpm_confidence, duration and multi-resolution flags, bit for bit.
* Escalation row reuse (hop-1024 frames and even hop-256 frames read from the hop-512
  spectrogram) against its control SDSP_NO_ROW_REUSE=1, which computes every
  escalation STFT frame: identical results, on ragged lengths whose (n - 2048) / 256 is odd and
  even and on tracks shorter than 2304 samples.
* Key spectrograms of 1 .. 300 frames around the mask margin and the HPCP tiles, peaks_per_frame
  8 / 16 / 32 list capacities, and a batch split into several sub-batches by a small HBM budget,
  against the oracle.
* Config-2/-5 shapes at a larger batch than the parity tests: 3-min tracks checked against the
  oracle on a sample.
"""
import numpy as np
import pytest

import oracle
import parity
import sdsp

pytestmark = pytest.mark.gpu


def _device_tracks(lens, seed0, bpm_mode=0):
    """Track i is the first lens[i] samples of synthetic track seed0 + i (one generator call, so
    bpm_mode 1 cycles through its three BPM ranges)."""
    lens = np.asarray(lens, dtype=np.uint64)
    Lmax = int(max(int(lens.max()), 1))
    buf = sdsp.DeviceBuffer(len(lens) * Lmax)
    sdsp.generate_synthetic(buf.ptr, len(lens), Lmax, seed0=seed0, bpm_mode=bpm_mode)
    offs = (np.arange(len(lens)) * Lmax).astype(np.uint64)
    return buf, offs, lens


def _bits(v):
    return np.float32(v).tobytes()


def test_bpm_only_equals_full():
    n, L = 36, 44100 * 45
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, seed0=900, bpm_mode=1)
    offs, lens = np.arange(n) * L, np.full(n, L)
    full = sdsp.analyze_batch_device(buf.ptr, offs, lens)
    bpm = sdsp.analyze_batch_device(buf.ptr, offs, lens, stages=sdsp.STAGES_BPM_ONLY)
    trig = 0
    for i, (a, b) in enumerate(zip(full, bpm)):
        assert _bits(a["bpm"]) == _bits(b["bpm"]), i
        assert _bits(a["bpm_confidence"]) == _bits(b["bpm_confidence"]), i
        for k in ("duration_seconds", "tempogram_multi_res_triggered", "tempogram_multi_res_used",
                  "tempogram_percussive_triggered", "tempogram_percussive_used"):
            assert a["metadata"][k] == b["metadata"][k], (i, k)
        assert b["beat_grid"]["beats"] == [] and b["key_confidence"] == 0.0
        trig += a["metadata"]["tempogram_multi_res_triggered"] is True
    assert trig >= n // 3, trig


def test_bpm_only_errors_match_full():
    lens = [44100 * 20, 0, 1000, 44100 * 5]
    buf, offs, lens = _device_tracks(lens, 950)
    zeros = np.zeros(44100 * 5, np.float32)
    buf.from_host(zeros, int(offs[3]))  # an all-silent track
    full = sdsp.analyze_batch_device(buf.ptr, offs, lens)
    bpm = sdsp.analyze_batch_device(buf.ptr, offs, lens, stages=sdsp.STAGES_BPM_ONLY)
    for a, b in zip(full, bpm):
        if isinstance(a, sdsp.AnalysisError):
            assert isinstance(b, sdsp.AnalysisError) and (a.code, str(a)) == (b.code, str(b))
        else:
            assert _bits(a["bpm"]) == _bits(b["bpm"])


def _strip(r):
    if isinstance(r, sdsp.AnalysisError):
        return ("err", r.code, str(r))
    m = dict(r["metadata"])
    m.pop("processing_time_ms", None)
    return {k: v for k, v in r.items() if k != "metadata"} | {"metadata": m}


def test_row_reuse_matches_control(monkeypatch):
    # n - 2048 = 256 k + r: k odd and even (hop-256 frame count parity), plus sub-2304 tracks
    base = 44100 * 40
    lens = [base + 256 * k + r for k, r in [(0, 0), (1, 0), (2, 17), (3, 255), (10, 100), (11, 1)]]
    lens += [2300, 2303, 2304, 2305, 2048 + 256 * 3 + 5, 44100 * 25 + 256]
    buf, offs, lens = _device_tracks(lens, 1200, bpm_mode=1)
    monkeypatch.delenv("SDSP_NO_ROW_REUSE", raising=False)
    reuse = sdsp.analyze_batch_device(buf.ptr, offs, lens)
    monkeypatch.setenv("SDSP_NO_ROW_REUSE", "1")
    ctrl = sdsp.analyze_batch_device(buf.ptr, offs, lens)
    trig = 0
    for i, (a, b) in enumerate(zip(reuse, ctrl)):
        assert _strip(a) == _strip(b), (i, int(lens[i]))
        if not isinstance(a, sdsp.AnalysisError):
            trig += a["metadata"]["tempogram_multi_res_triggered"] is True
    assert trig >= 3, trig  # the switch is exercised on escalated tracks


def test_config2_sample_of_a_larger_batch():
    """64 device-generated 3-min tracks in one batch (3 sub-batches are not needed at this size,
    but the batch is 1/16 of config 2); 6 of them checked against the oracle, bit-exact."""
    n, L = 64, 44100 * 180
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, seed0=2000)
    res = sdsp.analyze_batch_device(buf.ptr, np.arange(n) * L, np.full(n, L))
    assert all(not isinstance(r, sdsp.AnalysisError) for r in res)
    for i in (0, 9, 21, 33, 47, 63):
        x = buf.to_host(i * L, L)
        st, ref = oracle.analyze(x, 44100)
        assert st == 0
        assert not parity.diff_results(res[i], ref), (i, parity.diff_results(res[i], ref))
        assert parity.exact_fraction(res[i], ref) == 1.0, i


def _key_frames_to_len(f8):
    """Samples of a track whose 8192/512 key spectrogram has f8 frames."""
    return 8192 + 512 * (f8 - 1) + 100


def test_key_frame_counts_around_tiles():
    """Key spectrograms of 1 .. 300 frames around the mask margin (12) and the HPCP tile (256), and
    3-min tracks, in one batch: every result equals the oracle's bit for bit."""
    f8s = [1, 2, 11, 12, 13, 15, 16, 17, 25, 26, 31, 32, 33, 255, 256, 257, 271, 272, 300]
    lens = [_key_frames_to_len(f) for f in f8s] + [44100 * 180, 44100 * 180 + 12345, 44100 * 37]
    buf, offs, lens = _device_tracks(lens, 1500)
    got = sdsp.analyze_batch_device(buf.ptr, offs, lens)
    for i in range(len(lens)):
        st, ref = oracle.analyze(buf.to_host(int(offs[i]), int(lens[i])), 44100)
        if st != 0:
            assert isinstance(got[i], sdsp.AnalysisError) and got[i].code == st, i
            continue
        assert parity.exact_fraction(got[i], ref) == 1.0 and not parity.diff_results(got[i], ref), i


@pytest.mark.parametrize("peaks", [8, 16, 32])
def test_key_peak_list_capacities(peaks):
    cfg = sdsp.default_config()
    cfg.key_hpcp_peaks_per_frame = peaks
    lens = [44100 * 30, 44100 * 61 + 7, _key_frames_to_len(40)]
    buf, offs, lens = _device_tracks(lens, 1600 + peaks)
    got = sdsp.analyze_batch_device(buf.ptr, offs, lens, config=cfg)
    for i in range(len(lens)):
        st, ref = oracle.analyze(buf.to_host(int(offs[i]), int(lens[i])), 44100, config=cfg)
        assert st == 0 and parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, i


@pytest.mark.parametrize("late_join", [True, False])
def test_sub_batches_vs_oracle(monkeypatch, late_join):
    """A batch split into several sub-batches by a small HBM budget (two streams), with the key
    results joined one sub-batch late (default: the key tail runs beside the next sub-batch's
    tempo path) and at the end of each sub-batch (SDSP_NO_KEY_DEFER=1): equal results, a sample
    against the oracle."""
    lens = [44100 * 30 + 37 * k for k in range(36)] + [5000, 44100 * 61]
    buf, offs, lens = _device_tracks(lens, 1700)
    monkeypatch.setenv("SDSP_HBM_BUDGET_GB", "1")  # several sub-batches
    if late_join:
        monkeypatch.delenv("SDSP_NO_KEY_DEFER", raising=False)
    else:
        monkeypatch.setenv("SDSP_NO_KEY_DEFER", "1")
    got = sdsp.analyze_batch_device(buf.ptr, offs, lens)
    assert sdsp.stage_times()["stft8192_launches"] >= 2
    for i in (0, 17, 35, 36, 37):
        st, ref = oracle.analyze(buf.to_host(int(offs[i]), int(lens[i])), 44100)
        assert st == 0 and parity.exact_fraction(got[i], ref) == 1.0, i
    # every track's result equals the other join's
    monkeypatch.setenv("SDSP_NO_KEY_DEFER", "1")
    ctl = sdsp.analyze_batch_device(buf.ptr, offs, lens)
    for i, (a, b) in enumerate(zip(got, ctl)):
        assert not parity.diff_results(a, b) and parity.exact_fraction(a, b, strict=True) == 1.0, i
