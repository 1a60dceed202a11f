"""Edge inputs of the default path, GPU engine against the oracle (empty, ragged, maximum
and non-finite inputs as the domain has them).  Each case either fails in both with the same
AnalysisError (kind and text) or gives results equal within the north-star tolerances and
bit-identical (tests/parity.py), NaN / inf propagation included:

* sample rates other than 44.1 kHz (the frame rate, mel and chroma bin edges, tolerances in
  samples all move with it);
* DC offset, a full-scale clipped square wave, a single impulse in silence, white noise;
* non-finite samples (NaN, +-inf inside an otherwise normal track; the reference's peak
  normalisation, silence detection and STFT all see them);
* samples of subnormal scale (everything below the silence threshold).
"""
import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu


def _same(x, sr, cfg=None):
    st, ref = oracle.analyze(x, sr, cfg)
    if st != 0:
        with pytest.raises(sdsp.AnalysisError) as ei:
            sdsp.analyze_audio(x, sr, config=cfg)
        assert ei.value.code == st and str(ei.value) == ref, (ei.value.code, str(ei.value), st, ref)
        return None
    got = sdsp.analyze_audio(x, sr, config=cfg)
    bad = parity.diff_results(got, ref)
    assert not bad, bad
    assert parity.exact_fraction(got, ref) == 1.0
    return got


@pytest.mark.parametrize("sr", [8000, 22050, 32000, 48000, 96000])
def test_sample_rates(sr):
    x, *_ = synth.make_track(7100 + sr % 97, seconds=16.0, sr=sr)
    assert _same(x, sr) is not None


def test_dc_offset():
    x, *_ = synth.make_track(7200, seconds=15.0)
    _same((x * np.float32(0.5) + np.float32(0.4)).astype(np.float32), 44100)


def test_clipped_square_wave():
    t = np.arange(44100 * 12, dtype=np.float64) / 44100
    x = np.sign(np.sin(2 * np.pi * 2.0 * t)).astype(np.float32)  # 2 Hz full-scale square: 240 edges / min
    _same(x, 44100)


def test_single_impulse_in_silence():
    x = np.zeros(44100 * 10, np.float32)
    x[44100 * 4] = 0.9
    _same(x, 44100)


def test_white_noise():
    x = (np.random.default_rng(7300).standard_normal(44100 * 12) * 0.3).astype(np.float32)
    _same(x, 44100)


@pytest.mark.parametrize("bad", ["nan", "inf", "-inf"])
def test_non_finite_samples(bad):
    x, *_ = synth.make_track(7400, seconds=12.0)
    x = x.copy()
    v = {"nan": np.nan, "inf": np.inf, "-inf": -np.inf}[bad]
    x[[44100 * 3, 44100 * 3 + 17, 44100 * 8]] = np.float32(v)
    _same(x, 44100)


def test_subnormal_scale_samples():
    x, *_ = synth.make_track(7500, seconds=10.0)
    _same((x * np.float32(1e-39)).astype(np.float32), 44100)


def test_edge_batch_equals_single_calls():
    """The same edge inputs through one ragged batch: every slot equals its single call."""
    xs = [np.zeros(44100 * 3, np.float32), synth.make_track(7600, seconds=9.0)[0],
          (np.random.default_rng(7601).standard_normal(44100 * 5) * 0.2).astype(np.float32)]
    xs[0][44100] = 0.5
    outs = sdsp.analyze_batch(xs, 44100)
    for x, o in zip(xs, outs):
        st, ref = oracle.analyze(x, 44100)
        if st != 0:
            assert isinstance(o, sdsp.AnalysisError) and o.code == st, (o, st, ref)
        else:
            assert isinstance(o, dict) and not parity.diff_results(o, ref), parity.diff_results(o, ref)
