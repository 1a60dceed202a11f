"""The reference's own beat-tracking unit tests, restated against the CPU restatement
(oracle/units.py -> oracle/o_beat.cpp unit probes).  CPU only.

One test per reference #[test], same name, same inputs and assertions:
  src/features/beat_tracking/mod.rs:488-700             generate_beat_grid, downbeats, grid stability
  src/features/beat_tracking/bayesian.rs:291-420        BayesianBeatTracker
  src/features/beat_tracking/tempo_variation.rs:230-330 detect_tempo_variations, has_tempo_variation
  src/features/beat_tracking/time_signature.rs:202-285  detect_time_signature
Rust-only plumbing the reference also asserts (TimeSignature::beats_per_bar / name, the
tracker's getters) is restated on the oracle's (beats-per-bar, name) mapping.
"""
import numpy as np
import pytest

import units as U


def f32_seq(n, step, start=0.0):
    """(0..n).map(|i| i as f32 * step) in f32."""
    return [float(np.float32(i) * np.float32(step)) + start for i in range(n)]


# ---- beat_tracking/mod.rs ----
def test_generate_beat_grid_basic():
    beats, downs, bars, stab = U.generate_beat_grid(120.0, 0.85, [0.0, 0.5, 1.0, 1.5, 2.0, 2.5, 3.0, 3.5], 44100)
    assert beats
    assert 0.0 <= stab <= 1.0
    assert all(beats[i] > beats[i - 1] for i in range(1, len(beats)))


def test_generate_beat_grid_128bpm():
    on = f32_seq(8, np.float32(60.0) / np.float32(128.0))
    beats, _, _, stab = U.generate_beat_grid(128.0, 0.8, on, 44100)
    assert beats and stab > 0.0


def test_generate_beat_grid_invalid_bpm():
    for bpm in (0.0, 350.0):
        with pytest.raises(U.AnalysisError):
            U.generate_beat_grid(bpm, 0.8, [0.0, 0.5, 1.0], 44100)


def test_generate_beat_grid_empty_onsets():
    with pytest.raises(U.AnalysisError):
        U.generate_beat_grid(120.0, 0.8, [], 44100)


def test_detect_downbeats():
    d = U.detect_downbeats([0.0, 0.5, 1.0, 1.5, 2.0, 2.5, 3.0, 3.5, 4.0], 120.0)
    assert d and d[0] == 0.0
    if len(d) > 1:
        assert abs((d[1] - d[0]) - 2.0) < 0.3


def test_detect_downbeats_empty():
    assert U.detect_downbeats([], 120.0) == []


def test_detect_downbeats_single_beat():
    assert U.detect_downbeats([0.5], 120.0) == [0.5]


def test_calculate_grid_stability_perfect():
    assert U.calculate_grid_stability([0.0, 0.5, 1.0, 1.5], 120.0) > 0.9


def test_calculate_grid_stability_variable():
    s = U.calculate_grid_stability([0.0, 0.4, 0.9, 1.6], 120.0)
    assert s < 0.9 and 0.0 <= s <= 1.0


def test_calculate_grid_stability_insufficient_beats():
    assert U.calculate_grid_stability([0.0], 120.0) == 0.0


def test_generate_beat_grid_from_positions():
    # generate_beat_grid_from_positions (mod.rs:264-320): sorted beats, 4/4 downbeats, bars = downbeats
    times = [0.0, 0.5, 1.0, 1.5, 2.0]
    beats = sorted(times)
    downs = U.detect_downbeats(beats, 120.0, 4)
    bars = list(downs)
    assert len(beats) == 5
    assert downs
    assert len(bars) == len(downs)


def test_generate_beat_grid_from_positions_empty():
    # the reference rejects an empty position list before downbeat detection (mod.rs:290-295);
    # the oracle's full grid path rejects empty onsets the same way
    with pytest.raises(U.AnalysisError):
        U.generate_beat_grid(120.0, 0.8, [], 44100)


# ---- bayesian.rs ----
def test_bayesian_tracker_creation():
    t = U.BayesianBeatTracker(120.0, 0.8)
    assert t.current_bpm == 120.0
    assert t.current_confidence == np.float32(0.8)
    assert t.history == [120.0]


def test_bayesian_tracker_confidence_clamping():
    assert U.BayesianBeatTracker(120.0, 1.5).current_confidence == 1.0
    assert U.BayesianBeatTracker(120.0, -0.5).current_confidence == 0.0


def test_generate_bpm_candidates():
    c = U.BayesianBeatTracker(120.0, 0.8).generate_bpm_candidates()
    assert c
    assert any(abs(b - 120.0) < 0.1 for b in c)
    assert min(c) >= 115.0 and max(c) <= 125.0


def test_compute_likelihood():
    t = U.BayesianBeatTracker(120.0, 0.8)
    on = [0.0, 0.5, 1.0, 1.5, 2.0]
    lik = t.compute_likelihood(on, 120.0)
    assert 0.0 < lik <= 1.0
    assert lik > t.compute_likelihood(on, 100.0)


def test_compute_likelihood_empty_onsets():
    assert U.BayesianBeatTracker(120.0, 0.8).compute_likelihood([], 120.0) == 0.0


def test_compute_prior():
    t = U.BayesianBeatTracker(120.0, 0.8)
    p = t.compute_prior(120.0)
    assert 0.0 < p <= 1.0
    assert p > t.compute_prior(130.0)


def test_update_with_onsets():
    t = U.BayesianBeatTracker(120.0, 0.8)
    bpm, conf = t.update_with_onsets([0.0, 0.5, 1.0, 1.5, 2.0], 44100)
    assert bpm > 0.0 and 0.0 <= conf <= 1.0
    assert t.current_bpm == bpm and t.current_confidence == conf
    assert len(t.history) == 2


def test_update_with_onsets_empty():
    with pytest.raises(U.AnalysisError):
        U.BayesianBeatTracker(120.0, 0.8).update_with_onsets([], 44100)


def test_update_with_onsets_invalid_bpm():
    for bpm in (0.0, 350.0):
        with pytest.raises(U.AnalysisError):
            U.BayesianBeatTracker(bpm, 0.8).update_with_onsets([0.0, 0.5], 44100)


def test_get_bpm_and_confidence():
    t = U.BayesianBeatTracker(120.0, 0.85)
    assert t.current_bpm == 120.0 and t.current_confidence == np.float32(0.85)


def test_get_history():
    t = U.BayesianBeatTracker(120.0, 0.8)
    t.update_with_onsets([0.0, 0.5, 1.0], 44100)
    assert len(t.history) == 2 and t.history[0] == 120.0


# ---- tempo_variation.rs ----
def test_detect_tempo_variations_constant():
    segs = U.detect_tempo_variations(f32_seq(20, np.float32(60.0) / np.float32(120.0)), 120.0)
    assert segs
    assert not U.has_tempo_variation(segs)


def test_detect_tempo_variations_variable():
    beats, t = [], np.float32(0.0)
    for i in range(20):
        t = np.float32(t + np.float32(60.0) / (np.float32(120.0) + np.float32(i) * np.float32(1.0)))
        beats.append(float(t))
    assert U.detect_tempo_variations(beats, 120.0)


def test_detect_tempo_variations_insufficient_beats():
    segs = U.detect_tempo_variations([0.0, 0.5, 1.0], 120.0)
    assert len(segs) == 1 and segs[0][2] == 120.0


def test_detect_tempo_variations_empty():
    segs = U.detect_tempo_variations([], 120.0)
    assert len(segs) == 1 and segs[0][2] == 120.0


def test_has_tempo_variation():
    segs = [(0.0, 4.0, 120.0, 0.8, False), (4.0, 8.0, 130.0, 0.6, True)]
    assert U.has_tempo_variation(segs)
    assert not U.has_tempo_variation([(0.0, 4.0, 120.0, 0.8, False)])


# ---- time_signature.rs ----
def beats_at(n, interval):
    out, t = [], np.float32(0.0)
    for _ in range(n):
        out.append(float(t))
        t = np.float32(t + np.float32(interval))
    return out


def test_time_signature_four_four():
    bpb, conf = U.detect_time_signature(beats_at(16, 0.5), 120.0)
    assert 0.0 <= conf <= 1.0
    assert bpb in (4, 3, 6)


def test_time_signature_three_four():
    _, conf = U.detect_time_signature(beats_at(12, 0.5), 120.0)
    assert 0.0 <= conf <= 1.0


def test_time_signature_insufficient_beats():
    assert U.detect_time_signature([0.0, 0.5, 1.0, 1.5], 120.0) == (4, 0.5)


SIGNATURES = {4: "4/4", 3: "3/4", 6: "6/8"}  # TimeSignature::{FourFour, ThreeFour, SixEight}


def test_time_signature_beats_per_bar():
    assert sorted(SIGNATURES) == [3, 4, 6]


def test_time_signature_name():
    assert (SIGNATURES[4], SIGNATURES[3], SIGNATURES[6]) == ("4/4", "3/4", "6/8")
