"""The oracle's legacy BPM estimator (oracle/o_period.cpp: legacy_autocorr, legacy_comb,
merge_candidates, estimate_bpm_legacy), pinned to the reference's own unit tests:
autocorrelation.rs:345-465, comb_filter.rs:404-543, candidate_filter.rs:450-590, restated on the
same inputs with the same assertions.  These are the checker for the GPU legacy path
(k_legacy.hip, force_legacy_bpm / enable_bpm_fusion)."""
import numpy as np

import oracle

f32 = np.float32
GUARD = [72.0, 168.0, 60.0, 210.0, 1.30, 0.70, 0.01]  # AnalysisConfig::default() (config.rs)


def _beats_frames(bpm, n=4, sr=44100, hop=512):
    period = f32(60.0 * sr) / f32(bpm)
    pf = int(np.round(period / f32(hop)))
    return [b * pf * hop for b in range(n)]


def _beats_samples(bpm, n=4, sr=44100):
    period = f32(60.0 * sr) / f32(bpm)
    return [int(np.round(f32(b) * period)) for b in range(n)]


# ---- autocorrelation.rs tests ----

def test_autocorrelation_120_128():
    for bpm in (120.0, 128.0):
        c = oracle.legacy("autocorr", _beats_frames(bpm), min_bpm=60.0, max_bpm=180.0)
        assert c and abs(c[0][0] - bpm) < 5.0 and c[0][1] > 0.0, (bpm, c[:3])


def test_autocorrelation_edge_cases():
    assert oracle.legacy("autocorr", [], min_bpm=60.0, max_bpm=180.0) < 0
    assert oracle.legacy("autocorr", [1000], min_bpm=60.0, max_bpm=180.0) == []
    assert oracle.legacy("autocorr", [1000, 2000], sample_rate=0, min_bpm=60.0, max_bpm=180.0) < 0
    assert oracle.legacy("autocorr", [1000, 2000], hop=0, min_bpm=60.0, max_bpm=180.0) < 0
    assert oracle.legacy("autocorr", [1000, 2000], min_bpm=180.0, max_bpm=60.0) < 0


# ---- comb_filter.rs tests ----

def test_comb_120_128():
    for bpm in (120.0, 128.0):
        c = oracle.legacy("comb", _beats_samples(bpm), min_bpm=60.0, max_bpm=180.0, res=1.0)
        assert c and abs(c[0][0] - bpm) < 5.0 and c[0][1] > 0.0, (bpm, c[:3])


def test_comb_edge_cases():
    assert oracle.legacy("comb", [], min_bpm=60.0, max_bpm=180.0) < 0
    assert oracle.legacy("comb", [1000], min_bpm=60.0, max_bpm=180.0) == []
    assert oracle.legacy("comb", [1000, 2000], sample_rate=0, min_bpm=60.0, max_bpm=180.0) < 0
    assert oracle.legacy("comb", [1000, 2000], min_bpm=180.0, max_bpm=60.0) < 0
    assert oracle.legacy("comb", [1000, 2000], min_bpm=60.0, max_bpm=180.0, res=0.0) < 0


def test_comb_resolution():
    on = _beats_samples(120.0)
    c1 = oracle.legacy("comb", on, min_bpm=60.0, max_bpm=180.0, res=1.0)
    c05 = oracle.legacy("comb", on, min_bpm=60.0, max_bpm=180.0, res=0.5)
    assert len(c05) >= len(c1)


# ---- candidate_filter.rs tests ----

def test_merge_agreement():
    m = oracle.legacy("merge", autocorr=[(120.0, 0.9)], comb=[(120.0, 0.85)])
    assert m and abs(m[0][0] - 120.0) < 1.0 and m[0][1] > 0.9 and m[0][2] == 2


def test_merge_octave_errors():
    for a in (240.0, 60.0):
        m = oracle.legacy("merge", autocorr=[(a, 0.8)], comb=[(120.0, 0.9)])
        assert m and abs(m[0][0] - 120.0) < 1.0, (a, m)


def test_merge_grouping_empty_single_sorted():
    m = oracle.legacy("merge", autocorr=[(120.0, 0.8), (121.0, 0.7)], comb=[(120.5, 0.85)])
    assert len(m) == 1 and abs(m[0][0] - 120.0) < 2.0 and m[0][2] == 3
    assert oracle.legacy("merge") == []
    m = oracle.legacy("merge", autocorr=[(120.0, 0.8)])
    assert m[0][2] == 1 and f32(m[0][1]) <= f32(0.8)
    m = oracle.legacy("merge", autocorr=[(120.0, 0.9), (130.0, 0.7)], comb=[(120.0, 0.85)])
    assert all(m[i - 1][1] >= m[i][1] for i in range(1, len(m)))


# ---- the estimate on a regular onset train (not a reference test: a sanity range) ----

def test_estimate_regular_train():
    for bpm in (96.0, 120.0, 128.0, 150.0):
        on = _beats_samples(bpm, n=40)
        for g in (GUARD, None):  # the legacy estimator lands in the metrical family (it is not exact)
            e = oracle.legacy("estimate", on, guardrails=g)
            assert e and min(abs(e[0][0] - m * bpm) for m in (0.5, 1.0, 2.0)) < 3.0, (bpm, g, e)
