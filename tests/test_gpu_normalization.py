"""RMS and LUFS normalization on the GPU path against the oracle.

The gain is folded per track in sample order by k_loudness_gain (one lane per track): the RMS
sum of squares, or the K-weighting biquad with the gated 400-ms block loudness.  Cases: loud
tracks where the clip limit bites, quiet ones where the full gain applies, a track whose every
LUFS block is under the gate (the peak-normalization fallback), tracks shorter than one block,
ragged lengths (so tracks start at every 16-B misalignment inside the batch buffer), a 48-kHz
track, the reference fixtures, and the too-low sample rate error.
"""
import os

import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
METHODS = {"rms": 1, "lufs": 2}


def _cfgs(method):
    c = sdsp.default_config()
    c.normalization = METHODS[method]
    o = oracle.default_config()
    o.normalization = METHODS[method]
    return c, o


def _batch():
    xs = []
    for i, (seed, sec, amp) in enumerate(((1, 20.0, 1.0), (2, 17.3, 0.02), (3, 12.1, 3.0), (4, 9.7, 0.3))):
        x = synth.make_track(seed, seconds=sec)[0] * np.float32(amp)
        xs.append(x[: x.size - i].astype(np.float32))  # ragged: every start misalignment
    t = np.arange(44100 * 6, dtype=np.float32) / np.float32(44100)
    xs.append((np.sin(t * np.float32(2 * np.pi * 220)) * np.float32(2e-5)).astype(np.float32))  # under the gate
    xs.append(synth.make_track(7, seconds=15.0)[0][:30001])  # shorter than one LUFS block + change
    return xs


@pytest.mark.parametrize("method", sorted(METHODS))
def test_batch_parity(method):
    cfg, ocfg = _cfgs(method)
    xs = _batch()
    got = sdsp.analyze_batch(xs, 44100, cfg)
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, ocfg)
        if st != 0:
            assert isinstance(got[i], sdsp.AnalysisError) and str(got[i]) == ref, (method, i, got[i], ref)
            continue
        assert not isinstance(got[i], Exception), (method, i, got[i])
        bad = parity.diff_results(got[i], ref)
        assert not bad, f"{method} track {i}: {bad}"
        assert parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, (method, i)


@pytest.mark.parametrize("method", sorted(METHODS))
@pytest.mark.parametrize("name", ["120bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"])
def test_fixture_parity(method, name):
    x, sr = parity.load_wav(os.path.join(GOLDEN, name))
    cfg, ocfg = _cfgs(method)
    st, ref = oracle.analyze(x, sr, ocfg)
    assert st == 0
    assert not parity.diff_results(sdsp.analyze_audio(x, sr, cfg), ref)


def test_48k_and_changes_result():
    x = synth.make_track(9, seconds=14.0, sr=48000)[0] * np.float32(0.05)
    outs = {}
    for m in sorted(METHODS):
        cfg, ocfg = _cfgs(m)
        st, ref = oracle.analyze(x, 48000, ocfg)
        assert st == 0
        got = sdsp.analyze_audio(x, 48000, cfg)
        assert not parity.diff_results(got, ref), m
        outs[m] = got
    outs["peak"] = sdsp.analyze_audio(x, 48000)
    # the gains differ, so some float field moves between the three methods
    sig = {k: (v["bpm_confidence"], v["key_clarity"], v["grid_stability"]) for k, v in outs.items()}
    assert len(set(sig.values())) >= 2, sig


@pytest.mark.parametrize("sr", [16003, 22050])
def test_odd_block_lengths(sr):
    """16003 Hz: a 6401-sample LUFS block, so block ends fall at every phase of the 16-B loads."""
    xs = [synth.make_track(s, seconds=11.0, sr=sr)[0][: 11 * sr - s] for s in (12, 13, 14)]
    for m in sorted(METHODS):
        cfg, ocfg = _cfgs(m)
        got = sdsp.analyze_batch(xs, sr, cfg)
        for i, x in enumerate(xs):
            st, ref = oracle.analyze(x, sr, ocfg)
            assert st == 0 and not parity.diff_results(got[i], ref), (sr, m, i)


def test_lufs_low_sample_rate_error():
    cfg, ocfg = _cfgs("lufs")
    x = np.ones(5000, np.float32) * np.float32(0.1)
    st, ref = oracle.analyze(x, 2, ocfg)
    assert st == 1
    with pytest.raises(sdsp.AnalysisError) as ei:
        sdsp.analyze_audio(x, 2, cfg)
    assert ei.value.code == st and str(ei.value) == ref
