"""Known-answer tests of the CPU restatement (oracle/) against the reference's own exact unit
tests (SURVEY.md §8c "What pins results").  CPU only.

  consensus.rs:293-477            vote_onsets clustering / votes / confidences / errors
  tempogram_fft.rs:298-314        find_best_bpm_fft
  tempogram_autocorr.rs:285-301   find_best_bpm_autocorr (same selection rule)
  hmm.rs:457-498                  HMM state space and transition matrix
  templates.rs:291-303            each template's maximum is its tonic
  result.rs:272-365               key names and numerals (host-side binding, sdsp_abi)
"""
import numpy as np
import pytest

import oracle
import sdsp_abi

W4 = [0.25, 0.25, 0.25, 0.25]


# ---- consensus.rs:293-477 ----
def test_consensus_basic():
    c = oracle.vote_onsets([[1000], [1000], [1000], [1000]], W4, 50, 44100)
    assert len(c) == 1
    t, voted, conf = c[0]
    assert t == 1000 and voted == 4 and abs(conf - 1.0) < 0.01


def test_consensus_clustering():
    c = oracle.vote_onsets([[1000], [1050], [980], [1020]], W4, 50, 44100)
    assert len(c) == 1 and c[0][1] == 4 and abs(c[0][2] - 1.0) < 0.01


def test_consensus_separate():
    c = oracle.vote_onsets([[1000, 50000], [1050, 50500], [980, 50200], [1020, 49900]], W4, 50, 44100)
    assert len(c) == 2 and c[0][1] == 4 and c[1][1] == 4


def test_consensus_partial():
    c = oracle.vote_onsets([[1000], [1050], [], []], [0.3, 0.3, 0.2, 0.2], 50, 44100)
    assert len(c) == 1 and c[0][1] == 2 and abs(c[0][2] - 0.6) < 0.01


def test_consensus_weighted():
    c = oracle.vote_onsets([[1000], [], [], []], [0.5, 0.2, 0.2, 0.1], 50, 44100)
    assert len(c) == 1 and c[0][1] == 1 and abs(c[0][2] - 0.5) < 0.01


def test_consensus_empty():
    assert oracle.vote_onsets([[], [], [], []], W4, 50, 44100) == []


def test_consensus_sorted_by_confidence():
    c = oracle.vote_onsets([[1000, 20000, 50000], [1050, 20050, 50500], [980, 20100], [1020, 19950]], W4, 50, 44100)
    assert len(c) >= 2 and c[0][1] == 4
    assert all(c[i][2] <= c[i - 1][2] for i in range(1, len(c)))


def test_consensus_invalid_parameters():
    assert oracle.vote_onsets([[1000], [], [], []], W4, 50, 0) == -1       # sample rate 0
    assert oracle.vote_onsets([[1000], [], [], []], W4, 0, 44100) == -1     # tolerance 0
    assert oracle.vote_onsets([[1000], [], [], []], [-0.1, 0.25, 0.25, 0.25], 50, 44100) == -1


def test_consensus_time_conversion():
    c = oracle.vote_onsets([[44100], [], [], []], [1.0, 0.0, 0.0, 0.0], 50, 44100)
    assert len(c) == 1 and c[0][0] == 44100  # time_seconds = 44100 / 44100 = 1.0


# ---- tempogram_fft.rs / tempogram_autocorr.rs find_best ----
def test_find_best():
    bpm, val, conf = oracle.find_best([(120.0, 0.9), (60.0, 0.3), (180.0, 0.2)])
    assert bpm == 120.0
    assert val == np.float32(0.9)
    assert abs(conf - 2.0 / 3.0) < 1e-6


def test_find_best_empty():
    assert oracle.find_best([]) is None


# ---- hmm.rs:457-498 ----
def test_hmm_state_space():
    st, tr = oracle.hmm_model(120.0)
    for got, want in zip(st, [108.0, 114.0, 120.0, 126.0, 132.0]):
        assert abs(got - want) < 0.1
    assert tr.shape == (5, 5)
    assert all(tr[i, i] > 0.6 for i in range(5))
    assert all(tr[i, i + 1] > 0.1 and tr[i + 1, i] > 0.1 for i in range(4))
    assert tr[0, 4] == 0.0 and tr[4, 0] == 0.0
    np.testing.assert_allclose(tr.sum(axis=1), 1.0, atol=1e-6)


def test_hmm_track_regular_onsets():
    on = np.arange(0.0, 10.0, 0.5, dtype=np.float32)  # 120 BPM onsets
    beats = oracle.hmm_track(120.0, on)
    assert beats is not None and len(beats) == len(on)
    np.testing.assert_allclose(beats, on, atol=1e-5)
    assert oracle.hmm_track(0.0, on) is None and oracle.hmm_track(120.0, []) is None


# ---- templates.rs:291-303 ----
def test_templates_tonic_is_max():
    t = oracle.key_templates()
    for k in range(24):
        assert int(np.argmax(t[k])) == k % 12
        assert abs(float(np.linalg.norm(t[k])) - 1.0) < 1e-5


# ---- result.rs:272-365 (names / numerals of the binding's result mirror) ----
@pytest.mark.parametrize("tonic,name", [(0, "C"), (1, "C#"), (2, "D"), (6, "F#"), (11, "B")])
def test_key_name_major(tonic, name):
    assert sdsp_abi.key_name(0, tonic) == name


@pytest.mark.parametrize("tonic,name", [(0, "Cm"), (1, "C#m"), (2, "Dm"), (9, "Am"), (11, "Bm")])
def test_key_name_minor(tonic, name):
    assert sdsp_abi.key_name(1, tonic) == name


def test_key_numerical():
    major = {0: "1A", 7: "2A", 2: "3A", 9: "4A", 4: "5A", 11: "6A", 6: "7A", 1: "8A", 8: "9A", 3: "10A", 10: "11A",
             5: "12A"}
    minor = {9: "1B", 4: "2B", 11: "3B", 6: "4B", 1: "5B", 8: "6B", 3: "7B", 10: "8B", 5: "9B", 0: "10B", 7: "11B",
             2: "12B"}
    for t, s in major.items():
        assert sdsp_abi.key_numerical(0, t) == s
    for t, s in minor.items():
        assert sdsp_abi.key_numerical(1, t) == s


def test_key_from_numerical():
    assert sdsp_abi.key_from_numerical("1A") == (0, 0)
    assert sdsp_abi.key_from_numerical("2A") == (0, 7)
    assert sdsp_abi.key_from_numerical("7A") == (0, 6)
    assert sdsp_abi.key_from_numerical("12A") == (0, 5)
    assert sdsp_abi.key_from_numerical("1B") == (1, 9)
    assert sdsp_abi.key_from_numerical("2B") == (1, 4)
    assert sdsp_abi.key_from_numerical("10B") == (1, 0)
    for bad in ("0A", "13A", "1C", "", "A"):
        assert sdsp_abi.key_from_numerical(bad) is None
    for mode in (0, 1):
        for t in range(12):
            assert sdsp_abi.key_from_numerical(sdsp_abi.key_numerical(mode, t)) == (mode, t)
