"""The default key path against an independent float64 reading of the
Rust (tests/ref64.py: harmonic_mask64, hpcp64, smooth_chroma64, key_weights64,
detect_key_weighted64, key_path64), from a front end that shares nothing with the CPU restatement
but the trim bounds: float64 peak normalisation and a numpy-FFT 8192 / 512 STFT
(ref64.normalize_peak64, ref64.stft64).  CPU only.

References: src/lib.rs:961-1540 (the key block: mask, HPCP, smoothing, frame weights, segment
voting, clarity), src/features/chroma/extractor.rs:529-680, 1097-1150, 1246-1349,
src/features/chroma/smoothing.rs:37-94, src/features/key/detector.rs:68-313,
src/features/key/key_clarity.rs:51-93, src/features/key/templates.rs:64-140, the defaults of
src/config.rs:669-739.  The oracle and the HIP kernels agree bit for bit on these fields (the HIP
key energies within 1e-4), so this ties the GPU key path to a second reading.

Tolerances: the key equal; key_confidence and key_clarity within 1e-4 (the north star's); the
number of voting segments equal.  A segment whose clarity lies within 1e-4 of the 0.2 threshold
may vote in one reading and not the other (ref64.Ties records it); none of these inputs has one.
Measured: key equal on all 20, clarity within 5.6e-5.
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
_cache = {}


def _run(kind, what):
    key = (kind, str(what))
    if key not in _cache:
        if kind == "fixture":
            x, sr = parity.load_wav(os.path.join(HERE, "golden", what))
        else:
            x, *_ = synth.make_track(what[0], seconds=what[1])
            sr = 44100
        st, r, tr = oracle.analyze(x, sr, trace=True)
        assert st == 0, r
        xt = ref64.normalize_peak64(x)[tr["trim_start"]:tr["trim_end"]]
        ties = ref64.Ties()
        got = ref64.key_path64(ref64.stft64(xt, 8192, 512), sr, ties=ties)
        _cache[key] = (r, tr, got, list(ties))
    return _cache[key]


def _key_index(k):
    return k["Major"] if "Major" in k else 12 + k["Minor"]


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_key_path_float64(kind, what):
    r, tr, (key, conf, clarity), ties = _run(kind, what)
    if ties:
        return  # a segment at the clarity threshold: which segments vote is f32 rounding's call
    assert key == _key_index(r["key"]), (key, r["key"])
    assert abs(conf - r["key_confidence"]) <= 1e-4, (conf, r["key_confidence"])
    assert abs(clarity - r["key_clarity"]) <= 1e-4, (clarity, r["key_clarity"])


def test_key_path_coverage():
    """Both detection forms run (segment voting on the longer tracks, the whole-slice detection on
    the 4-bar fixtures), weights are used, and several different keys come out."""
    keys, voted, whole = set(), 0, 0
    for kind, what in CASES:
        r, tr, (key, conf, clarity), ties = _run(kind, what)
        keys.add(key)
        voted += tr["used_segments"] > 0
        whole += tr["used_segments"] == 0
        assert tr["weights_used"]
    assert voted >= 8 and whole >= 2 and len(keys) >= 6


def test_key_templates_match_oracle():
    """The float64 reading's Krumhansl-Kessler templates are the oracle's (to f32 rounding)."""
    maj, mnr = ref64.key_templates64()
    t = np.asarray(oracle.key_templates(), np.float64).reshape(-1, 12)
    assert np.max(np.abs(np.vstack([maj, mnr]) - t[:24])) <= 1e-6
