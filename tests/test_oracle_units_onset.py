"""The reference's own onset and silence unit tests, restated against the CPU restatement
(oracle/units.py -> oracle/o_onset.cpp unit probes).  CPU only.

One test per reference #[test], same name, same inputs and assertions:
  src/features/onset/energy_flux.rs:247-420    detect_energy_flux_onsets
  src/features/onset/spectral_flux.rs:225-372  detect_spectral_flux_onsets
  src/features/onset/hfc.rs:219-368            detect_hfc_onsets
  src/preprocessing/silence.rs:282-470         detect_and_trim
The performance test (energy_flux.rs test_energy_flux_performance, a 200 ms wall-clock bound)
is restated as the same call on the same 30-s input with the same bound.
"""
import time

import numpy as np
import pytest

import units as U


def kick_pattern(duration_s, bpm, sr, kick_ms):
    """energy_flux.rs:253-283 generate_kick_pattern (f32 arithmetic as in the reference)."""
    f32 = np.float32
    n = int(f32(duration_s) * f32(sr))
    x = np.zeros(n, np.float32)
    interval = int(f32(60.0) / f32(bpm) * f32(sr))
    ks = int(f32(kick_ms) / f32(1000.0) * f32(sr))
    env = np.array([np.exp(-(f32(i) / f32(ks)) * f32(5.0)) for i in range(ks)], np.float32)
    pos = 0
    while pos < n:
        end = min(pos + ks, n)
        x[pos:end] = env[:end - pos] * f32(0.8)
        pos += interval
    return x


# ---- energy_flux.rs ----
def test_energy_flux_basic():
    x = np.zeros(44100, np.float32)
    x[5000:] = 0.5
    on = U.detect_energy_flux_onsets(x, 2048, 512, -30.0)
    assert on, "Should detect at least one onset for step function"
    assert 3000 <= on[0] <= 8000


def test_energy_flux_kick_pattern_120_bpm():
    x = kick_pattern(4.0, 120.0, 44100.0, 150.0)
    on = U.detect_energy_flux_onsets(x, 2048, 512, -30.0)
    assert 6 <= len(on) <= 20
    if len(on) >= 2:
        expected = int(np.float32(60.0 / 120.0) * np.float32(44100.0))
        iv = np.diff(on)
        avg = int(iv.sum()) // len(iv)
        assert abs(avg - expected) < expected // 2


def test_energy_flux_empty_samples():
    assert U.detect_energy_flux_onsets([], 2048, 512, -20.0) == []


def test_energy_flux_silent_audio():
    assert U.detect_energy_flux_onsets(np.zeros(44100), 2048, 512, -20.0) == []


def test_energy_flux_too_short_audio():
    assert U.detect_energy_flux_onsets(np.full(1000, 0.5), 2048, 512, -20.0) == []


def test_energy_flux_invalid_parameters():
    x = np.full(44100, 0.5, np.float32)
    with pytest.raises(U.AnalysisError):
        U.detect_energy_flux_onsets(x, 0, 512, -20.0)
    with pytest.raises(U.AnalysisError):
        U.detect_energy_flux_onsets(x, 2048, 0, -20.0)


def test_energy_flux_threshold_sensitivity():
    x = kick_pattern(2.0, 120.0, 44100.0, 50.0)
    lo = U.detect_energy_flux_onsets(x, 2048, 512, -30.0)
    hi = U.detect_energy_flux_onsets(x, 2048, 512, -10.0)
    assert len(lo) >= len(hi)


def test_energy_flux_performance():
    x = kick_pattern(30.0, 120.0, 44100.0, 50.0)
    t0 = time.perf_counter()
    U.detect_energy_flux_onsets(x, 2048, 512, -20.0)
    assert time.perf_counter() - t0 <= 0.2


# ---- spectral_flux.rs ----
def spec_const(frames, bins, v):
    return [np.full(bins, v, np.float32) for _ in range(frames)]


def test_spectral_flux_basic():
    s = spec_const(10, 1024, 0.01)
    for i in range(5):
        s[i][:256] = 1.0
    s[5][768:1024] = 1.0
    for i in range(6, 10):
        s[i][:256] = 1.0
    on = U.detect_spectral_flux_onsets(s, 0.3)
    assert on
    assert any(4 <= f <= 7 for f in on), on


def test_spectral_flux_empty():
    assert U.detect_spectral_flux_onsets([], 0.8) == []


def test_spectral_flux_single_frame():
    assert U.detect_spectral_flux_onsets(spec_const(1, 1024, 0.5), 0.8) == []


def test_spectral_flux_invalid_percentile():
    s = spec_const(10, 1024, 0.5)
    for p in (-0.1, 1.5):
        with pytest.raises(U.AnalysisError):
            U.detect_spectral_flux_onsets(s, p)


def test_spectral_flux_inconsistent_lengths():
    s = spec_const(10, 1024, 0.5)
    s[5] = np.full(512, 0.5, np.float32)
    with pytest.raises(U.AnalysisError) as e:
        U.detect_spectral_flux_onsets(s, 0.8)
    assert e.value.kind == "InvalidInput"


def test_spectral_flux_all_zeros():
    on = U.detect_spectral_flux_onsets(spec_const(10, 1024, 0.0), 0.8)
    assert len(on) < 3


def test_spectral_flux_threshold_sensitivity():
    s = spec_const(20, 1024, 0.1)
    for i in range(20):
        s[i][:] = np.float32(0.1) + (np.float32(i) / np.float32(20.0)) * np.float32(0.9)
    lo = U.detect_spectral_flux_onsets(s, 0.5)
    hi = U.detect_spectral_flux_onsets(s, 0.9)
    assert len(lo) >= len(hi)


def test_spectral_flux_normalization():
    s = spec_const(2, 1024, 0.5)
    s[1] = np.full(1024, 1.0, np.float32)
    U.detect_spectral_flux_onsets(s, 0.5)  # must not fail


def test_spectral_flux_multiple_changes():
    s = spec_const(20, 1024, 0.1)
    s[5][:512] = 1.0
    s[10][512:1024] = 1.0
    s[15][256:768] = 1.0
    on = U.detect_spectral_flux_onsets(s, 0.3)
    assert len(on) >= 2, on


# ---- hfc.rs ----
def test_hfc_basic():
    s = spec_const(10, 1024, 0.01)
    for i in range(5):
        s[i][:100] = 0.5
    s[5][800:1024] = 1.0
    for i in range(6, 10):
        s[i][:100] = 0.5
    on = U.detect_hfc_onsets(s, 44100, 0.3)
    assert on
    assert any(4 <= f <= 7 for f in on), on


def test_hfc_empty():
    assert U.detect_hfc_onsets([], 44100, 0.8) == []


def test_hfc_single_frame():
    assert U.detect_hfc_onsets(spec_const(1, 1024, 0.5), 44100, 0.8) == []


def test_hfc_invalid_percentile():
    s = spec_const(10, 1024, 0.5)
    for p in (-0.1, 1.5):
        with pytest.raises(U.AnalysisError):
            U.detect_hfc_onsets(s, 44100, p)


def test_hfc_zero_sample_rate():
    with pytest.raises(U.AnalysisError):
        U.detect_hfc_onsets(spec_const(10, 1024, 0.5), 0, 0.8)


def test_hfc_inconsistent_lengths():
    s = spec_const(10, 1024, 0.5)
    s[5] = np.full(512, 0.5, np.float32)
    with pytest.raises(U.AnalysisError):
        U.detect_hfc_onsets(s, 44100, 0.8)


def test_hfc_all_zeros():
    assert U.detect_hfc_onsets(spec_const(10, 1024, 0.0), 44100, 0.8) == []


def test_hfc_threshold_sensitivity():
    s = spec_const(20, 1024, 0.01)
    for i in range(20):
        s[i][800:1024] = np.float32(0.1) + (np.float32(i) / np.float32(20.0)) * np.float32(0.9)
    lo = U.detect_hfc_onsets(s, 44100, 0.5)
    hi = U.detect_hfc_onsets(s, 44100, 0.9)
    assert len(lo) >= len(hi)


def test_hfc_frequency_weighting():
    s = spec_const(2, 1024, 0.0)
    s[0][:100] = 1.0
    s[1][900:1024] = 1.0
    U.detect_hfc_onsets(s, 44100, 0.5)  # must not fail


def test_hfc_multiple_changes():
    s = spec_const(20, 1024, 0.01)
    for f in (5, 10, 15):
        s[f][800:1024] = 1.0
    on = U.detect_hfc_onsets(s, 44100, 0.3)
    assert len(on) >= 2, on


# ---- preprocessing/silence.rs ----
def audio_with_silence(total, start, end, amp):
    """silence.rs:286-301: amplitude * sin(i / 1000) over [start, end)."""
    x = np.zeros(total, np.float32)
    i = np.arange(start, min(end, total))
    x[i] = np.float32(amp) * np.sin((i.astype(np.float32) / np.float32(1000.0)).astype(np.float32)).astype(np.float32)
    return x


def test_detect_and_trim_leading_trailing():
    x = audio_with_silence(44100 * 3, 44100, 44100 * 2, 0.5)
    trimmed, smap = U.detect_and_trim(x, 44100)
    assert len(trimmed) < len(x)
    assert len(trimmed) > 0
    assert smap


def test_detect_and_trim_all_silent():
    trimmed, _ = U.detect_and_trim(np.zeros(44100), 44100)
    assert len(trimmed) == 0 or np.all(np.abs(trimmed) < 1e-6)


def test_detect_and_trim_no_silence():
    x = audio_with_silence(44100, 0, 44100, 0.5)
    trimmed, _ = U.detect_and_trim(x, 44100, threshold_db=-60.0)
    assert len(trimmed) > len(x) // 2


def test_detect_and_trim_invalid_parameters():
    x = np.full(44100, 0.5, np.float32)
    with pytest.raises(U.AnalysisError):
        U.detect_and_trim(x, 0)
    with pytest.raises(U.AnalysisError):
        U.detect_and_trim(x, 44100, frame_size=0)


def test_detect_and_trim_empty_samples():
    trimmed, smap = U.detect_and_trim([], 44100)
    assert len(trimmed) == 0 and smap == []


def test_detect_and_trim_threshold_sensitivity():
    x = np.zeros(44100 * 2, np.float32)
    x[:22050] = 0.01
    x[22050:44100] = 0.5
    _, lo = U.detect_and_trim(x, 44100, threshold_db=-60.0)
    _, hi = U.detect_and_trim(x, 44100, threshold_db=-20.0)
    assert sum(e - s for s, e in hi) >= sum(e - s for s, e in lo)


def test_detect_and_trim_min_duration():
    x = np.full(44100 * 2, 0.5, np.float32)
    x[10000:15000] = 0.0
    U.detect_and_trim(x, 44100, min_duration_ms=500)  # must not fail
