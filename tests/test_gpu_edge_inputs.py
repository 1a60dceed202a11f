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
    assert parity.exact_fraction(got, ref, cfg=cfg) == 1.0
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


# Leading / trailing silence of assorted lengths: the trim start moves the energy pass's frames
# onto the raw signal's hop grid (launch_frame_rms_from_raw takes them from the trim pass), and
# the trimmed end cuts the last frames short (those are folded from the samples).
@pytest.mark.parametrize("lead,tail", [(0.0, 0.0), (0.37, 0.0), (1.3, 0.71), (2.9, 1.93), (0.0, 2.5)])
def test_leading_trailing_silence(lead, tail):
    sr = 44100
    x, *_ = synth.make_track(7400 + int(lead * 100) + int(tail * 10), seconds=14.0, sr=sr)
    y = np.concatenate([np.zeros(int(lead * sr), np.float32), x,
                        np.zeros(int(tail * sr) + 123, np.float32)]).astype(np.float32)
    assert _same(y, sr) is not None


def test_short_island_after_trimming():
    # ~1.5 frames of tone between long silences: the trimmed track is shorter than two frames
    sr = 44100
    y = np.zeros(sr * 6, np.float32)
    t = np.arange(3100, dtype=np.float64) / sr
    y[sr * 3 + 17: sr * 3 + 17 + 3100] = (0.5 * np.sin(2 * np.pi * 440.0 * t)).astype(np.float32)
    _same(y, sr)


@pytest.mark.parametrize("hop", [256, 384, 1024])
def test_trim_with_other_hops(hop):
    # hop 256 / 1024: the shared raw pass (G = 8 / 2); 384 does not divide the trim hop: two passes
    sr = 44100
    x, *_ = synth.make_track(7500 + hop, seconds=12.0, sr=sr)
    y = np.concatenate([np.zeros(int(1.7 * sr), np.float32), x, np.zeros(sr, np.float32)]).astype(np.float32)
    ocfg, cfg = oracle.default_config(), sdsp.default_config()
    ocfg.hop_size = cfg.hop_size = hop
    st, ref = oracle.analyze(y, sr, ocfg)
    assert st == 0
    got = sdsp.analyze_audio(y, sr, config=cfg)
    assert not parity.diff_results(got, ref)
    assert parity.exact_fraction(got, ref, cfg=cfg) == 1.0


def test_batch_mixed_trims():
    sr = 44100
    tracks, refs = [], []
    for k, lead in enumerate([0.0, 0.5, 1.25, 2.0]):
        x, *_ = synth.make_track(7600 + k, seconds=10.0 + k, sr=sr)
        y = np.concatenate([np.zeros(int(lead * sr), np.float32), x, np.zeros(int(0.3 * k * sr), np.float32)])
        tracks.append(y.astype(np.float32))
        st, ref = oracle.analyze(tracks[-1], sr)
        assert st == 0
        refs.append(ref)
    got = sdsp.analyze_batch(tracks, sr)
    for g, r in zip(got, refs):
        assert not parity.diff_results(g, r)
        assert parity.exact_fraction(g, r) == 1.0
