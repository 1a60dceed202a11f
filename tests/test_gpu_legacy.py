"""Parity of the legacy BPM paths (force_legacy_bpm, enable_bpm_fusion).

The legacy estimator (estimate_bpm_with_guardrails / estimate_bpm, src/features/period/mod.rs:196-404:
FFT autocorrelation of the onset train, comb filter, candidate merge, guardrails) runs on the GPU in
k_legacy.hip; force_legacy_bpm takes its estimate instead of the tempogram's, enable_bpm_fusion keeps
the tempogram BPM and moves its confidence (src/lib.rs:814-892).  Every result field is compared
with the oracle (oracle/o_period.cpp, pinned by tests/test_oracle_legacy.py) on the same inputs:
bit-exact.
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

_TRACKS = None


def tracks():
    """Synthetic device tracks (30 s, default and escalation-heavy BPM mixes; one 5-min track: a
    2^17-point ACF), host tracks, the reference fixtures and short tracks."""
    global _TRACKS
    if _TRACKS is None:
        xs = []
        for mode, seed in ((0, 40), (1, 700)):
            n, L = 4, 44100 * 30
            buf = sdsp.DeviceBuffer(n * L)
            sdsp.generate_synthetic(buf.ptr, n, L, seed0=seed, bpm_mode=mode)
            host = buf.to_host()
            xs += [host[i * L:(i + 1) * L].copy() for i in range(n)]
        buf = sdsp.DeviceBuffer(44100 * 300)
        sdsp.generate_synthetic(buf.ptr, 1, 44100 * 300, seed0=77)
        xs.append(buf.to_host())
        xs.append(synth.make_track(3, seconds=20.0)[0])
        for name in ("120bpm_4bar.wav", "128bpm_4bar.wav", "mixed_silence.wav"):
            xs.append(parity.load_wav(os.path.join(GOLDEN, name))[0])
        rng = np.random.default_rng(5)
        xs.append((rng.standard_normal(5000) * 0.3).astype(np.float32))
        xs.append((rng.standard_normal(44100) * 0.3).astype(np.float32))
        _TRACKS = xs
    return _TRACKS


def _apply(cfg, opts):
    for k, v in opts.items():
        setattr(cfg, k, v)
    return cfg


CASES = {
    "force": dict(force_legacy_bpm=1),
    "force_noguard": dict(force_legacy_bpm=1, enable_legacy_bpm_guardrails=0),
    "force_range": dict(force_legacy_bpm=1, min_bpm=60.0, max_bpm=200.0, bpm_resolution=0.5),
    "force_guard_custom": dict(force_legacy_bpm=1, legacy_bpm_preferred_min=150.0, legacy_bpm_preferred_max=90.0,
                               legacy_bpm_conf_mul_soft=0.2),
    "fusion": dict(enable_bpm_fusion=1),
    "fusion_noguard_cands": dict(enable_bpm_fusion=1, enable_legacy_bpm_guardrails=0, emit_tempogram_candidates=1),
    "fusion_no_multires": dict(enable_bpm_fusion=1, enable_tempogram_multi_resolution=0),
}


@pytest.mark.parametrize("case", list(CASES))
def test_legacy_parity(case):
    xs = tracks()
    cfg = _apply(sdsp.default_config(), CASES[case])
    ocfg = _apply(oracle.default_config(), CASES[case])
    got = sdsp.analyze_batch(xs, 44100, cfg)
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, ocfg)
        if st != 0:
            assert isinstance(got[i], sdsp.AnalysisError) and got[i].code == st, (case, i, got[i], ref)
            assert str(got[i]) == ref, (case, i)
            continue
        assert not isinstance(got[i], Exception), (case, i, got[i])
        bad = parity.diff_results(got[i], ref)
        assert not bad, f"{case} track {i}: {bad}"
        assert parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, (case, i)
        assert got[i]["bpm"] == ref["bpm"] and got[i]["bpm_confidence"] == ref["bpm_confidence"], (case, i)


def test_legacy_paths_live():
    """force_legacy_bpm changes some BPMs and clears the tempogram flags; fusion keeps every
    tempogram BPM and changes some confidences."""
    xs = tracks()
    base = sdsp.analyze_batch(xs, 44100, sdsp.default_config())
    force = sdsp.analyze_batch(xs, 44100, _apply(sdsp.default_config(), CASES["force"]))
    fusion = sdsp.analyze_batch(xs, 44100, _apply(sdsp.default_config(), CASES["fusion"]))
    moved = conf_moved = 0
    for b, f, u in zip(base, force, fusion):
        if not isinstance(b, dict):
            continue
        moved += b["bpm"] != f["bpm"]
        assert f["metadata"]["tempogram_multi_res_triggered"] is None
        assert u["bpm"] == b["bpm"]
        conf_moved += u["bpm_confidence"] != b["bpm_confidence"]
    assert moved >= 1 and conf_moved >= 1, (moved, conf_moved)
