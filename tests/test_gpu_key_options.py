"""Parity of the opt-in key-scoring branches against the oracle.

Each case switches on one branch of the reference's key path (src/lib.rs:1200-1470) -- chroma
sharpening, edge trim, Temperley templates, the K-K/Temperley ensemble, the mode heuristic and
minor leading-tone bonus (detector.rs:326-506), multi-scale voting (detector.rs:546-719) -- or a
combination, runs a ragged batch through the C ABI and compares every result field with the oracle
on the same inputs (bit-exact key, BPM within 1e-4).  The reference's own tests hold no golden
vectors for these branches: parity is against the CPU restatement (oracle/o_key.cpp), which follows
the reference file:line cited there.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu

TEMPERLEY = 1  # sdsp_template_set


def _tracks():
    out = []
    for seed, sec, mode in ((3, 30.0, 1), (11, 24.0, 0), (17, 40.0, 1), (29, 12.0, None), (41, 60.0, 0)):
        out.append(synth.make_track(seed, seconds=sec, mode=mode)[0])
    return out


_TRACKS = None


def tracks():
    global _TRACKS
    if _TRACKS is None:
        _TRACKS = _tracks()
    return _TRACKS


def _apply(cfg, opts, keep):
    for k, v in opts.items():
        if k in ("key_multi_scale_lengths", "key_multi_scale_weights"):
            arr = np.ascontiguousarray(v, dtype=np.uint64 if k.endswith("lengths") else np.float32)
            keep.append(arr)
            ct = C.c_uint64 if k.endswith("lengths") else C.c_float
            setattr(cfg, k, arr.ctypes.data_as(C.POINTER(ct)))
            setattr(cfg, k + "_len", arr.size)
        else:
            setattr(cfg, k, v)
    return cfg


CASES = {
    "sharpen2": dict(chroma_sharpening_power=2.0),
    "sharpen1.5": dict(chroma_sharpening_power=1.5),
    "edge_trim": dict(enable_key_edge_trim=1),
    "edge_trim_0.3": dict(enable_key_edge_trim=1, key_edge_trim_fraction=0.3),
    "temperley": dict(key_template_set=TEMPERLEY),
    "ensemble": dict(enable_key_ensemble=1),
    "ensemble_skew": dict(enable_key_ensemble=1, key_ensemble_kk_weight=0.8, key_ensemble_temperley_weight=0.3),
    "mode_heuristic": dict(enable_key_mode_heuristic=1),
    "minor_bonus": dict(enable_key_minor_harmonic_bonus=1),
    "heuristic_bonus_loose": dict(enable_key_mode_heuristic=1, enable_key_minor_harmonic_bonus=1,
                                  key_mode_third_ratio_margin=0.0, key_mode_flip_min_score_ratio=0.5,
                                  key_minor_leading_tone_bonus_weight=1.0),
    "heuristic_no_voting": dict(enable_key_mode_heuristic=1, enable_key_minor_harmonic_bonus=1,
                                enable_key_segment_voting=0, enable_key_frame_weighting=0),
    "multi_scale": dict(enable_key_multi_scale=1),
    "multi_scale_weighted": dict(enable_key_multi_scale=1, key_multi_scale_lengths=[90, 0, 300, 5000],
                                 key_multi_scale_weights=[1.0, 1.0, 0.5], key_multi_scale_hop=45),
    "multi_scale_heuristic": dict(enable_key_multi_scale=1, enable_key_mode_heuristic=1,
                                  enable_key_minor_harmonic_bonus=1, key_multi_scale_min_clarity=0.0),
    "multi_scale_none_pass": dict(enable_key_multi_scale=1, key_multi_scale_min_clarity=1.0),
    "combined": dict(chroma_sharpening_power=2.0, enable_key_edge_trim=1, key_template_set=TEMPERLEY,
                     enable_key_mode_heuristic=1, key_segment_min_clarity=0.0),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_key_option_parity(case):
    keep = []
    cfg = _apply(sdsp.default_config(), CASES[case], keep)
    ocfg = _apply(oracle.default_config(), CASES[case], keep)
    xs = tracks()
    got = sdsp.analyze_batch(xs, 44100, cfg)
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, ocfg)
        assert st == 0, (case, i, ref)
        assert not isinstance(got[i], Exception), (case, i, got[i])
        bad = parity.diff_results(got[i], ref)
        assert not bad, f"{case} track {i}: {bad}"
        assert parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, (case, i)
    # single-track API through the same path
    g1 = sdsp.analyze_audio(xs[0], 44100, cfg)
    assert not parity.diff_results(g1, oracle.analyze(xs[0], 44100, ocfg)[1])


def test_key_options_change_results():
    """The branches are live: across the cases some key result differs from the default config."""
    xs = tracks()
    base = sdsp.analyze_batch(xs, 44100, sdsp.default_config())
    changed = set()
    for case in ("sharpen2", "temperley", "ensemble", "heuristic_bonus_loose", "multi_scale", "edge_trim"):
        keep = []
        got = sdsp.analyze_batch(xs, 44100, _apply(sdsp.default_config(), CASES[case], keep))
        for a, b in zip(got, base):
            if (a["key"], a["key_confidence"], a["key_clarity"]) != (b["key"], b["key_confidence"], b["key_clarity"]):
                changed.add(case)
    assert len(changed) >= 5, changed
