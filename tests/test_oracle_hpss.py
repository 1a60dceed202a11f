"""The oracle's HPSS restatement (oracle/o_onset.cpp: hpss_decompose, hpss_onsets).

Pinned two ways:
- the reference's own unit tests for src/features/onset/hpss.rs (:380-532), restated on the
  same inputs with the same assertions;
- a numpy float32 restatement of hpss.rs:71-281 / :275-373 written independently here (sorted
  windows, IEEE f32 arithmetic), compared bit-exactly on random and structured spectrograms.
The reference holds no golden vectors for HPSS, so beyond those unit tests the values are
"parity unpinned" upstream: the numpy restatement is a second reading of the same source.
"""
import numpy as np
import pytest

import oracle

f32 = np.float32


def _median_rows(w):
    # hpss.rs:195-202: sort the window, even length -> mean of the middle two (times 0.5)
    n = w.shape[0]
    s = np.sort(w, axis=0)
    if n % 2:
        return s[n // 2]
    return (s[n // 2 - 1] + s[n // 2]) * f32(0.5)


def np_hpss(m, margin):
    m = np.asarray(m, f32)
    F, B = m.shape
    H, P = m.copy(), m.copy()
    for it in range(10):
        hp, pp = H.copy(), P.copy()
        hf = np.empty_like(m)
        pf = np.empty_like(m)
        for t in range(F):  # apply_horizontal_median_filter (:179-209)
            hf[t] = _median_rows(H[max(t - margin, 0):min(t + margin + 1, F)])
        for b in range(B):  # apply_vertical_median_filter (:213-243)
            pf[:, b] = _median_rows(P[:, max(b - margin, 0):min(b + margin + 1, B)].T)
        total = hf + pf
        ok = total > f32(1e-10)
        with np.errstate(divide="ignore", invalid="ignore"):
            H = np.where(ok, m * (hf / total), m * f32(0.5)).astype(f32)
            P = np.where(ok, m * (pf / total), m * f32(0.5)).astype(f32)
        if it > 0:
            ch = max(np.abs(H - hp).max(initial=f32(0)), np.abs(P - pp).max(initial=f32(0)))
            if ch < f32(1e-6):
                break
    return H, P


def np_hpss_onsets(p, pct):
    p = np.asarray(p, f32)
    if p.shape[0] == 0:
        return []
    if not (0.0 <= pct <= 1.0):
        return None
    if p.shape[0] < 2:
        return []
    e = np.empty(p.shape[0], f32)
    for t in range(p.shape[0]):  # sequential f32 sum of squares (:305-308)
        s = f32(0)
        for v in p[t]:
            s = f32(s + f32(v * v))
        e[t] = s
    flux = np.maximum(e[1:] - e[:-1], f32(0))
    srt = np.sort(flux)
    idx = min(int(f32(len(srt)) * f32(pct)), len(srt) - 1)
    thr = srt[idx]
    on = [i + 1 for i in range(1, len(flux) - 1) if flux[i] > thr and flux[i] > flux[i - 1] and flux[i] >= flux[i + 1]]
    if len(flux) > 1 and flux[0] > thr and flux[0] >= flux[1]:
        on.append(1)
    L = len(flux) - 1
    if len(flux) > 1 and flux[L] > thr and flux[L] > flux[L - 1]:
        on.append(len(flux))
    return sorted(set(on))


# ---- the reference's unit tests (hpss.rs:380-532) ----

def test_hpss_decompose_basic():
    m = np.full((10, 1024), 0.5, f32)
    st, h, p = oracle.hpss(m, 5)
    assert st == 0 and h.shape == m.shape and p.shape == m.shape
    assert np.abs((h + p) - m).max() < 0.1


def test_hpss_decompose_empty():
    st, _, _ = oracle.hpss(np.zeros((0, 1024), f32), 5)
    assert st != 0
    st, _, _ = oracle.hpss(np.zeros((10, 0), f32), 5)
    assert st != 0


def test_hpss_decompose_harmonic_vs_percussive():
    m = np.zeros((20, 1024), f32)
    m[:, 100:200] = 0.8
    m[[5, 10, 15], :] = 1.0
    st, _, p = oracle.hpss(m, 3)
    assert st == 0
    assert (p[5] ** 2).sum() > (p[3] ** 2).sum()


def test_detect_hpss_onsets_basic():
    p = np.full((20, 1024), 0.01, f32)
    p[[5, 10, 15], :] = 1.0
    on = oracle.hpss_onsets(p, 0.5)
    assert on is not None and len(on) >= 2


def test_detect_hpss_onsets_empty_and_single():
    assert oracle.hpss_onsets(np.zeros((0, 1024), f32), 0.8) == []
    assert oracle.hpss_onsets(np.full((1, 1024), 0.5, f32), 0.8) == []


def test_detect_hpss_onsets_invalid_percentile():
    p = np.full((10, 1024), 0.5, f32)
    assert oracle.hpss_onsets(p, -0.1) is None
    assert oracle.hpss_onsets(p, 1.5) is None


def test_detect_hpss_onsets_threshold_sensitivity():
    p = np.full((20, 1024), 0.01, f32)
    for i in range(20):
        p[i, :] = f32(0.1) + (f32(i) / f32(20.0)) * f32(0.9)
    assert len(oracle.hpss_onsets(p, 0.5)) >= len(oracle.hpss_onsets(p, 0.9))


# ---- bit-exact cross-check against the numpy restatement ----

def _specs():
    rng = np.random.default_rng(7)
    yield "random", rng.random((37, 61), dtype=np.float32)
    s = np.zeros((50, 80), f32)
    s[:, 10:20] = 0.8
    s[[7, 21, 33], :] = 1.0
    s += rng.random(s.shape, dtype=np.float32) * f32(0.05)
    yield "structured", s
    yield "tiny", rng.random((3, 5), dtype=np.float32)
    z = np.zeros((12, 30), f32)
    z[4, 3] = 1e-12  # below the soft-mask floor
    yield "near_zero", z
    q = np.round(rng.random((25, 40), dtype=np.float32) * 4) / f32(4)  # many ties
    yield "ties", q.astype(f32)


@pytest.mark.parametrize("margin", [0, 1, 3, 10, 16])
def test_hpss_matches_numpy(margin):
    for name, s in _specs():
        st, h, p = oracle.hpss(s, margin)
        assert st == 0
        H, P = np_hpss(s, margin)
        assert np.array_equal(h, H), (name, margin)
        assert np.array_equal(p, P), (name, margin)
        for pct in (0.0, 0.5, 0.8, 1.0):
            assert oracle.hpss_onsets(p, pct) == np_hpss_onsets(P, pct), (name, margin, pct)
