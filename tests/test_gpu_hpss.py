"""Parity of the HPSS branches (HPSS onsets and the percussive tempogram fallback).

- `enable_hpss_onsets` (src/lib.rs:222-236): hpss_decompose of the hop-512 spectrogram
  (hpss.rs:71-172) and detect_hpss_onsets (:275-373) as the fourth consensus list.
- `enable_tempogram_percussive_fallback` (src/lib.rs:582-683): for tracks in the low trap zone
  of the multi-resolution escalation, the tempogram re-run on the percussive component and the
  family-move acceptance rule.

Each case runs a ragged batch through the C ABI (GPU: k_hpss.hip) and compares every result field
and the escalation flags with the oracle (oracle/o_onset.cpp, o_analyze.cpp) on the same inputs:
bit-exact. The oracle's HPSS is pinned by tests/test_oracle_hpss.py.  Both outcomes of the
acceptance rule are exercised: the crafted chord-stab track (synth.chord_stab_track) makes it take
the percussive estimate (tempogram_percussive_used = true), the other trap-zone tracks do not.
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


def _kick_track(bpm, seconds, tone, sr=44100):
    """A 60 Hz kick (e^-10t, 100 ms) on every beat under a sustained triad: the tempogram stays at
    the kick rate, so low BPMs land in the trap zone [55, 80] and trigger the percussive fallback."""
    n = int(sr * seconds)
    x = np.zeros(n, np.float64)
    kt = np.arange(int(0.1 * sr)) / sr
    kick = np.sin(2 * np.pi * 60 * kt) * np.exp(-10 * kt)
    s = 0.0
    while s < seconds:
        i = int(s * sr)
        e = min(i + kick.size, n)
        x[i:e] += kick[:e - i]
        s += 60.0 / bpm
    t = np.arange(n) / sr
    x += tone * sum(np.sin(2 * np.pi * f * t) for f in (220.0, 277.18, 329.63)) / 3
    return (x * 0.9 / np.abs(x).max()).astype(np.float32)


def tracks():
    """12-s escalation-heavy synthetic mix (BASELINE config 5 recipe), low-BPM kick tracks, a
    78 BPM synthetic track, the reference's 120 BPM fixture and short tracks (1 and 2 frames)."""
    global _TRACKS
    if _TRACKS is None:
        n, L = 6, 44100 * 12
        buf = sdsp.DeviceBuffer(n * L)
        sdsp.generate_synthetic(buf.ptr, n, L, seed0=500, bpm_mode=1)
        host = buf.to_host()
        xs = [host[i * L:(i + 1) * L].copy() for i in range(n)]
        xs.append(_kick_track(58.0, 12.0, 0.3))
        xs.append(_kick_track(70.0, 10.0, 0.1))
        xs.append(synth.make_track(9, seconds=8.0, bpm=78.0)[0])
        xs.append(synth.chord_stab_track())  # the percussive estimate is accepted (see synth.py)
        xs.append(parity.load_wav(os.path.join(GOLDEN, "120bpm_4bar.wav"))[0])
        rng = np.random.default_rng(3)
        xs.append((rng.standard_normal(2048) * 0.3).astype(np.float32))
        xs.append((rng.standard_normal(2600) * 0.3).astype(np.float32))
        _TRACKS = xs
    return _TRACKS


def _apply(cfg, opts):
    for k, v in opts.items():
        setattr(cfg, k, v)
    return cfg


CASES = {
    "hpss_onsets": dict(enable_hpss_onsets=1),
    "hpss_onsets_m3": dict(enable_hpss_onsets=1, hpss_margin=3),
    "hpss_onsets_m16_pct": dict(enable_hpss_onsets=1, hpss_margin=16, onset_threshold_percentile=0.6),
    "perc_fallback": dict(enable_tempogram_percussive_fallback=1),
    "perc_fallback_m5": dict(enable_tempogram_percussive_fallback=1, hpss_margin=5),
    "both": dict(enable_hpss_onsets=1, enable_tempogram_percussive_fallback=1),
    "both_cands": dict(enable_hpss_onsets=1, enable_tempogram_percussive_fallback=1, emit_tempogram_candidates=1),
}


@pytest.mark.parametrize("case", list(CASES))
def test_hpss_parity(case):
    xs = tracks()
    cfg = _apply(sdsp.default_config(), CASES[case])
    ocfg = _apply(oracle.default_config(), CASES[case])
    got = sdsp.analyze_batch(xs, 44100, cfg)
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, ocfg)
        if st != 0:
            assert isinstance(got[i], sdsp.AnalysisError) and got[i].code == st, (case, i, got[i], ref)
            continue
        assert not isinstance(got[i], Exception), (case, i, got[i])
        bad = parity.diff_results(got[i], ref)
        assert not bad, f"{case} track {i}: {bad}"
        assert parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, (case, i)
        m, rm = got[i]["metadata"], ref["metadata"]
        for k in ("tempogram_multi_res_triggered", "tempogram_multi_res_used", "tempogram_percussive_triggered",
                  "tempogram_percussive_used"):
            assert m[k] == rm[k], (case, i, k, m[k], rm[k])


def test_hpss_branches_live():
    """The fallback is triggered on trap-zone tracks and the HPSS list changes some result."""
    xs = tracks()
    got = sdsp.analyze_batch(xs, 44100, _apply(sdsp.default_config(), CASES["perc_fallback"]))
    trig = sum(1 for g in got if isinstance(g, dict) and g["metadata"]["tempogram_percussive_triggered"] is True)
    assert trig >= 2, trig
    # the acceptance rule's "taken" outcome (src/lib.rs:640-668) on the crafted chord-stab track
    used = [g for g in got if isinstance(g, dict) and g["metadata"]["tempogram_percussive_used"] is True]
    assert len(used) >= 1 and 140.0 < used[0]["bpm"] < 148.0, [g["bpm"] for g in used]
    base = sdsp.analyze_batch(xs, 44100, sdsp.default_config())
    on = sdsp.analyze_batch(xs, 44100, _apply(sdsp.default_config(), CASES["hpss_onsets"]))
    diff = 0
    for a, b in zip(base, on):
        if isinstance(a, dict) and isinstance(b, dict):
            diff += (a["beat_grid"], a["bpm_confidence"], a["grid_stability"]) != \
                (b["beat_grid"], b["bpm_confidence"], b["grid_stability"])
    assert diff >= 1, diff


def test_hpss_margin_limit():
    cfg = _apply(sdsp.default_config(), dict(enable_hpss_onsets=1, hpss_margin=17))
    with pytest.raises(sdsp.AnalysisError) as ei:
        sdsp.analyze_audio(tracks()[0], 44100, cfg)
    assert "hpss_margin" in str(ei.value)
