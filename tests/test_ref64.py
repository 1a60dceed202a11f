"""The CPU restatement (oracle/, C++, f32 in the reference's order) against an independent float64
restatement of the same reference functions (tests/ref64.py, numpy), stage by stage, on the
reference's 4 WAV fixtures and 16 seeded synthetic tracks.  CPU only.

Stages:
  a10-a13 novelty: the default band-fusion full novelty curve, elementwise within 1e-4
  a14-a16 tempogram estimate: BPM within 1e-4, confidence within 1e-4, agreement equal, and the
          first 5 scored candidates within 1e-4 (BPM) / 1e-4 (score); candidate BPMs are the
          reference's f32 grid values (discrete), so they match exactly
  a20-a23 beat grid: beat and downbeat times within 1e-4 s, stability within 1e-4, the tempo-
          variation / Bayesian branches equal
The oracle and the HIP kernels are bit-identical (tests/test_gpu_*.py), so this is what ties the
GPU path to a second, independent reading of the Rust.

Where the reference's own f32 rounding decides a comparison (relative margin < 1e-5 between the
two best Bayesian likelihoods or time-signature scores, or a zero-confidence tempogram tie), the
float64 reading cannot predict the reference's pick: ref64 records those near ties and the test
then checks that the oracle's pick is one of the tied options and compares everything up to the
tie.  The summary test bounds how often that happens.
"""
import os

import numpy as np
import pytest

import oracle
import parity
import ref64
import synth

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = ["120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"]
SYNTH = [(s, (20.0, 30.0, 45.0)[s % 3]) for s in range(16)]
CASES = [("fixture", n) for n in FIXTURES] + [("synth", s) for s in SYNTH]


def _load(kind, what):
    if kind == "fixture":
        return parity.load_wav(os.path.join(HERE, "golden", what))
    seed, sec = what
    x, *_ = synth.make_track(seed, seconds=sec)
    return x.astype(np.float32), 44100


_cache = {}


def _stage_inputs(kind, what):
    key = (kind, str(what))
    if key not in _cache:
        x, sr = _load(kind, what)
        st, r, tr = oracle.analyze(x, sr, trace=True)
        assert st == 0, r
        _, xn = oracle.normalize(x, 0, sr)  # peak, -1 dB (src/lib.rs:116-127)
        mags = oracle.stft(xn[tr["trim_start"]:tr["trim_end"]], 2048, 512)
        _cache[key] = (sr, r, tr, mags)
    return _cache[key]


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_novelty_full(kind, what):
    sr, _, _, mags = _stage_inputs(kind, what)
    a = oracle.novelty_full(mags, sr)
    b = ref64.novelty_full(mags.astype(np.float64))
    assert a.size == b.size
    assert np.max(np.abs(a - b)) <= 1e-4


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_tempogram_estimate(kind, what):
    sr, _, tr, mags = _stage_inputs(kind, what)
    bpm, conf, agree, scored = ref64.estimate_bpm_tempogram(mags.astype(np.float64), sr, 512, 40.0, 240.0, 1.0)
    obpm, oconf, oagree = tr["base"]

    def score64(b):  # ref64's score of the candidate at BPM b (candidate BPMs match within 1e-4)
        m = [c[1] for c in scored if abs(c[0] - b) <= 1e-4]
        assert m, ("candidate missing from the float64 reading", b)
        return m[0]

    ties = ref64.estimate_bpm_tempogram.lookup_ties

    def tied(b):
        return any(abs(t - b) <= 1e-4 for t in ties)

    # every top-5 candidate of the oracle is a float64 candidate with the same score, unless its
    # nearest-bin lookup is a tie that f32 rounding decides
    for c32 in tr["base_cands"][:5]:
        assert tied(c32[0]) or abs(score64(c32[0]) - c32[1]) <= 1e-4, c32
    if abs(bpm - obpm) > 1e-4:
        # the picks may differ only between candidates both readings score alike (a near tie that
        # f32 rounding decides, e.g. which of two candidates the >180 fold finds first)
        assert tied(obpm) or tied(bpm) or abs(score64(obpm) - score64(bpm)) <= 1e-4, (bpm, obpm)
        return
    assert abs(conf - oconf) <= 1e-4, (conf, oconf)
    assert agree == oagree


def _beat_compare(r, tr, sr):
    on = np.array(tr["chosen_onsets"], np.float64) / sr
    beats = np.array(r["beat_grid"]["beats"])
    if r["bpm"] <= 0 or on.size < 2:
        return None
    g = ref64.generate_beat_grid(r["bpm"], r["bpm_confidence"], on)
    assert g is not None
    b64, d64, stab, diag = g
    assert diag["variable"] == bool(tr["beat_variable"])
    assert diag["refined"] == bool(tr["beat_refined"])
    bayes_ties = [t[1] for t in diag["ties"] if t[0] == "bayes"]
    ts_ties = [t[1] for t in diag["ties"] if t[0] == "time_signature"]
    if bayes_ties:
        # the refined beats agree up to the first segment whose Bayesian argmax is a near tie
        cut = min(t for t in bayes_ties)
        a, b = np.array(b64), beats
        a, b = a[a < cut - 1.0], b[b < cut - 1.0]
        assert a.size == b.size and (a.size == 0 or np.max(np.abs(a - b)) <= 1e-4)
        return "bayes-tie"
    assert len(b64) == beats.size and (beats.size == 0 or np.max(np.abs(np.array(b64) - beats)) <= 1e-4)
    assert abs(stab - r["grid_stability"]) <= 1e-4
    bpb = tr["beats_per_bar"]
    if ts_ties:
        assert bpb in ts_ties[0]
        bar = (60.0 / r["bpm"]) * bpb  # downbeats with the oracle's pick of the tied signatures
        d64 = [b64[0]]
        for t in b64[1:]:
            if abs(t - (d64[-1] + bar)) <= bar * 0.1:
                d64.append(t)
    else:
        assert diag["beats_per_bar"] == bpb
    downs = np.array(r["beat_grid"]["downbeats"])
    assert len(d64) == downs.size and (downs.size == 0 or np.max(np.abs(np.array(d64) - downs)) <= 1e-4)
    return "ts-tie" if ts_ties else "exact"


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_beat_grid(kind, what):
    sr, r, tr, _ = _stage_inputs(kind, what)
    _beat_compare(r, tr, sr)


def test_branches_and_tie_rate():
    """The Bayesian refinement (mod.rs:152-219) is reached, and f32-decided near ties stay rare."""
    outcomes, refined = [], 0
    for kind, what in CASES:
        sr, r, tr, _ = _stage_inputs(kind, what)
        outcomes.append(_beat_compare(r, tr, sr))
        refined += bool(tr["beat_refined"])
    assert refined >= 1
    assert outcomes.count("exact") + outcomes.count("ts-tie") >= 0.75 * len([o for o in outcomes if o])


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_tempogram_estimate_float64_front_end(kind, what):
    """The tempogram estimate from a float64 front end that shares nothing with the CPU
    restatement but the trim bounds: peak normalisation and the STFT in float64 with numpy's FFT
    (ref64.normalize_peak64 / stft64), then ref64's novelty and tempogram.  The oracle's BPM (f32,
    the spec FFT) is the float64 pick, or a candidate the float64 reading scores within 1e-4 of
    it (a near tie decided by rounding)."""
    x, sr = _load(kind, what)
    _, _, tr, _ = _stage_inputs(kind, what)
    xt = ref64.normalize_peak64(x)[tr["trim_start"]:tr["trim_end"]]
    mags = ref64.stft64(xt, 2048, 512)
    bpm, conf, agree, scored = ref64.estimate_bpm_tempogram(mags, sr, 512, 40.0, 240.0, 1.0)
    obpm, oconf, oagree = tr["base"]
    if abs(bpm - obpm) <= 1e-4:
        assert abs(conf - oconf) <= 1e-4, (conf, oconf)
        return
    ties = ref64.estimate_bpm_tempogram.lookup_ties
    s64 = {round(c[0], 4): c[1] for c in scored}
    assert any(abs(t - obpm) <= 1e-4 for t in ties) or abs(s64.get(round(obpm, 4), -1.0) - s64[round(bpm, 4)]) <= 1e-4, (bpm, obpm)

