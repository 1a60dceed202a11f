"""The reference's own key / chroma unit tests, restated against the CPU restatement
(oracle/units.py -> oracle/o_key.cpp unit probes).  CPU only.

One test per reference #[test], same name, same inputs and assertions:
  src/features/key/detector.rs:1004-1075        detect_key / detect_key_weighted / dot_product
  src/features/key/key_clarity.rs:96-160        compute_key_clarity
  src/features/chroma/smoothing.rs:162-235      smooth_chroma / smooth_chroma_average
Key indices are mode * 12 + tonic (Major(0) = 0).
"""
import numpy as np
import pytest

import units as U


# ---- key/detector.rs ----
def test_detect_key_empty():
    with pytest.raises(U.AnalysisError):
        U.detect_key([])


def test_detect_key_basic():
    ch = np.zeros(12, np.float32)
    ch[[0, 4, 7]] = 0.3
    ch = (ch / np.float32(np.sqrt(np.float32((ch * ch).sum())))).astype(np.float32)
    key, conf, all_scores, top = U.detect_key([ch] * 10)
    assert 0.0 <= conf <= 1.0
    assert len(all_scores) == 24
    assert key == 0
    assert 0 < len(top) <= 3
    assert top[0][0] == 0


def test_detect_key_wrong_dimensions():
    with pytest.raises(U.AnalysisError):
        U.detect_key([np.zeros(10, np.float32)])


def test_average_chroma():
    U.detect_key_weighted([np.zeros(12, np.float32)] * 10, np.zeros(10, np.float32))  # must not fail


def test_dot_product():
    assert U.dot_product([1.0, 2.0, 3.0], [4.0, 5.0, 6.0]) == 32.0


# ---- key/key_clarity.rs ----
def test_compute_key_clarity_empty():
    assert U.compute_key_clarity([]) == 0.0


def test_compute_key_clarity_single():
    assert U.compute_key_clarity([(0, 0.8)]) == 0.0


def test_compute_key_clarity_high():
    assert U.compute_key_clarity([(0, 0.9), (1, 0.3), (2, 0.3), (3, 0.3)]) > 0.5


def test_compute_key_clarity_low():
    assert U.compute_key_clarity([(0, 0.5), (1, 0.48), (2, 0.49), (3, 0.47)]) < 0.5


def test_compute_key_clarity_all_same():
    assert U.compute_key_clarity([(0, 0.5), (1, 0.5), (2, 0.5)]) == 0.0


def test_compute_key_clarity_clamped():
    assert 0.0 <= U.compute_key_clarity([(0, 1.0), (1, 0.0)]) <= 1.0


# ---- chroma/smoothing.rs ----
def one_hot_frames(n):
    ch = np.zeros((n, 12), np.float32)
    for i in range(n):
        ch[i, i % 12] = 1.0
    return ch


def test_smooth_chroma_empty():
    assert len(U.smooth_chroma(np.zeros((0, 12), np.float32), 5)) == 0


def test_smooth_chroma_single_frame():
    s = U.smooth_chroma(np.full((1, 12), 0.1, np.float32), 5)
    assert s.shape == (1, 12)


def test_smooth_chroma_basic():
    s = U.smooth_chroma(one_hot_frames(10), 3)
    assert s.shape == (10, 12)


def test_smooth_chroma_window_size_one():
    x = np.full((5, 12), 0.1, np.float32)
    assert len(U.smooth_chroma(x, 1)) == len(x)


def test_smooth_chroma_average():
    s = U.smooth_chroma_average(one_hot_frames(10), 3)
    assert s.shape == (10, 12)


def test_smooth_chroma_even_window_size():
    assert len(U.smooth_chroma(np.full((10, 12), 0.1, np.float32), 4)) == 10
