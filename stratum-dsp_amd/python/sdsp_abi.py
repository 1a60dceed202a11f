"""ctypes mirror of include/stratum_hip.h (the C ABI of libstratum_hip.so).

Field order and types must match the header exactly; tests/test_abi.py checks sizes and
offsets against the compiled library (sdsp_abi_layout probe).
"""
import ctypes as C

u8, i8, i32, u32, u64, f32 = C.c_uint8, C.c_int8, C.c_int32, C.c_uint32, C.c_uint64, C.c_float


class SdspConfig(C.Structure):
    """AnalysisConfig, reference src/config.rs:8-592."""

    _fields_ = [
        ("min_amplitude_db", f32),
        ("normalization", i32),
        ("enable_normalization", u8),
        ("enable_silence_trimming", u8),
        ("enable_onset_consensus", u8),
        ("onset_threshold_percentile", f32),
        ("onset_consensus_tolerance_ms", u32),
        ("onset_consensus_weights", f32 * 4),
        ("enable_hpss_onsets", u8),
        ("hpss_margin", u64),
        ("force_legacy_bpm", u8),
        ("enable_bpm_fusion", u8),
        ("enable_legacy_bpm_guardrails", u8),
        ("enable_tempogram_multi_resolution", u8),
        ("tempogram_multi_res_top_k", u64),
        ("tempogram_multi_res_w512", f32),
        ("tempogram_multi_res_w256", f32),
        ("tempogram_multi_res_w1024", f32),
        ("tempogram_multi_res_structural_discount", f32),
        ("tempogram_multi_res_double_time_512_factor", f32),
        ("tempogram_multi_res_margin_threshold", f32),
        ("tempogram_multi_res_use_human_prior", u8),
        ("enable_tempogram_percussive_fallback", u8),
        ("enable_tempogram_band_fusion", u8),
        ("tempogram_band_low_max_hz", f32),
        ("tempogram_band_mid_max_hz", f32),
        ("tempogram_band_high_max_hz", f32),
        ("tempogram_band_w_full", f32),
        ("tempogram_band_w_low", f32),
        ("tempogram_band_w_mid", f32),
        ("tempogram_band_w_high", f32),
        ("tempogram_band_seed_only", u8),
        ("tempogram_band_support_threshold", f32),
        ("tempogram_band_consensus_bonus", f32),
        ("tempogram_novelty_w_spectral", f32),
        ("tempogram_novelty_w_energy", f32),
        ("tempogram_novelty_w_hfc", f32),
        ("tempogram_novelty_local_mean_window", u64),
        ("tempogram_novelty_smooth_window", u64),
        ("has_debug_track_id", u8),
        ("debug_track_id", u32),
        ("has_debug_gt_bpm", u8),
        ("debug_gt_bpm", f32),
        ("debug_top_n", u64),
        ("enable_tempogram_mel_novelty", u8),
        ("tempogram_mel_n_mels", u64),
        ("tempogram_mel_fmin_hz", f32),
        ("tempogram_mel_fmax_hz", f32),
        ("tempogram_mel_max_filter_bins", u64),
        ("tempogram_mel_weight", f32),
        ("tempogram_superflux_max_filter_bins", u64),
        ("emit_tempogram_candidates", u8),
        ("tempogram_candidates_top_n", u64),
        ("legacy_bpm_preferred_min", f32),
        ("legacy_bpm_preferred_max", f32),
        ("legacy_bpm_soft_min", f32),
        ("legacy_bpm_soft_max", f32),
        ("legacy_bpm_conf_mul_preferred", f32),
        ("legacy_bpm_conf_mul_soft", f32),
        ("legacy_bpm_conf_mul_extreme", f32),
        ("min_bpm", f32),
        ("max_bpm", f32),
        ("bpm_resolution", f32),
        ("frame_size", u64),
        ("hop_size", u64),
        ("center_frequency", f32),
        ("soft_chroma_mapping", u8),
        ("soft_mapping_sigma", f32),
        ("chroma_sharpening_power", f32),
        ("enable_key_spectrogram_time_smoothing", u8),
        ("key_spectrogram_smooth_margin", u64),
        ("enable_key_frame_weighting", u8),
        ("key_min_tonalness", f32),
        ("key_tonalness_power", f32),
        ("key_energy_power", f32),
        ("enable_key_harmonic_mask", u8),
        ("key_harmonic_mask_power", f32),
        ("enable_key_hpss_harmonic", u8),
        ("key_hpss_frame_step", u64),
        ("key_hpss_time_margin", u64),
        ("key_hpss_freq_margin", u64),
        ("key_hpss_mask_power", f32),
        ("enable_key_stft_override", u8),
        ("key_stft_frame_size", u64),
        ("key_stft_hop_size", u64),
        ("enable_key_log_frequency", u8),
        ("enable_key_beat_synchronous", u8),
        ("enable_key_multi_scale", u8),
        ("key_template_set", i32),
        ("enable_key_ensemble", u8),
        ("key_ensemble_kk_weight", f32),
        ("key_ensemble_temperley_weight", f32),
        ("enable_key_median", u8),
        ("key_median_segment_length_frames", u64),
        ("key_median_segment_hop_frames", u64),
        ("key_median_min_segments", u64),
        ("key_multi_scale_lengths", C.POINTER(u64)),
        ("key_multi_scale_lengths_len", u64),
        ("key_multi_scale_hop", u64),
        ("key_multi_scale_min_clarity", f32),
        ("key_multi_scale_weights", C.POINTER(f32)),
        ("key_multi_scale_weights_len", u64),
        ("enable_key_tuning_compensation", u8),
        ("key_tuning_max_abs_semitones", f32),
        ("key_tuning_frame_step", u64),
        ("key_tuning_peak_rel_threshold", f32),
        ("enable_key_edge_trim", u8),
        ("key_edge_trim_fraction", f32),
        ("enable_key_segment_voting", u8),
        ("key_segment_len_frames", u64),
        ("key_segment_hop_frames", u64),
        ("key_segment_min_clarity", f32),
        ("enable_key_mode_heuristic", u8),
        ("key_mode_third_ratio_margin", f32),
        ("key_mode_flip_min_score_ratio", f32),
        ("enable_key_hpcp", u8),
        ("key_hpcp_peaks_per_frame", u64),
        ("key_hpcp_num_harmonics", u64),
        ("key_hpcp_harmonic_decay", f32),
        ("key_hpcp_mag_power", f32),
        ("enable_key_hpcp_whitening", u8),
        ("key_hpcp_whitening_smooth_bins", u64),
        ("enable_key_hpcp_bass_blend", u8),
        ("key_hpcp_bass_fmin_hz", f32),
        ("key_hpcp_bass_fmax_hz", f32),
        ("key_hpcp_bass_weight", f32),
        ("enable_key_minor_harmonic_bonus", u8),
        ("key_minor_leading_tone_bonus_weight", f32),
        ("enable_ml_refinement", u8),
    ]


class SdspTempoCandidate(C.Structure):
    _fields_ = [("bpm", f32), ("score", f32), ("fft_norm", f32), ("autocorr_norm", f32), ("selected", u8)]


class SdspResult(C.Structure):
    """AnalysisResult + metadata, reference src/analysis/result.rs:144-263."""

    _fields_ = [
        ("bpm", f32),
        ("bpm_confidence", f32),
        ("key_mode", i32),
        ("key_tonic", u32),
        ("key_confidence", f32),
        ("key_clarity", f32),
        ("beats", C.POINTER(f32)),
        ("n_beats", u64),
        ("downbeats", C.POINTER(f32)),
        ("n_downbeats", u64),
        ("bars", C.POINTER(f32)),
        ("n_bars", u64),
        ("grid_stability", f32),
        ("duration_seconds", f32),
        ("sample_rate", u32),
        ("processing_time_ms", f32),
        ("algorithm_version", C.c_char * 16),
        ("onset_method_consensus", f32),
        ("methods_used", u32),
        ("flags", u32),
        ("warnings", C.POINTER(C.c_char_p)),
        ("n_warnings", u64),
        ("tempogram_candidates", C.POINTER(SdspTempoCandidate)),
        ("n_tempogram_candidates", u64),
        ("has_tempogram_candidates", i8),
        ("tempogram_multi_res_triggered", i8),
        ("tempogram_multi_res_used", i8),
        ("tempogram_percussive_triggered", i8),
        ("tempogram_percussive_used", i8),
        ("status", i32),
        ("error_message", C.c_char * 256),
    ]


class SdspStageTimes(C.Structure):
    _fields_ = [
        ("stft2048_ms", C.c_double),
        ("stft8192_ms", C.c_double),
        ("features_ms", C.c_double),
        ("tempogram_ms", C.c_double),
        ("key_ms", C.c_double),
        ("beat_ms", C.c_double),
        ("total_ms", C.c_double),
        ("stft2048_launches", u64),
        ("stft8192_launches", u64),
        ("stft2048_bytes", C.c_double),
        ("stft8192_bytes", C.c_double),
        ("stft2048_frames", u64),
        ("stft8192_frames", u64),
        ("key_reruns", u64),
        ("rerun_ms", C.c_double),
    ]


class SdspConfidence(C.Structure):
    _fields_ = [
        ("bpm_confidence", f32),
        ("key_confidence", f32),
        ("grid_stability", f32),
        ("overall_confidence", f32),
        ("n_flags", u32),
        ("flag_list", C.c_int32 * 8),
    ]


NOTE_NAMES = ["C", "C#", "D", "D#", "E", "F", "F#", "G", "G#", "A", "A#", "B"]
FLAG_NAMES = ["MultimodalBpm", "WeakTonality", "TempoVariation", "OnsetDetectionAmbiguous"]
ERROR_NAMES = {1: "InvalidInput", 2: "DecodingError", 3: "ProcessingError", 4: "NotImplemented", 5: "NumericalError"}


def key_name(mode, tonic):
    """Key::name, result.rs:30-39."""
    return NOTE_NAMES[tonic % 12] + ("m" if mode == 1 else "")


def key_numerical(mode, tonic):
    """Key::numerical, result.rs:59-87."""
    maj = [0, 7, 2, 9, 4, 11, 6, 1, 8, 3, 10, 5]
    mnr = [9, 4, 11, 6, 1, 8, 3, 10, 5, 0, 7, 2]
    tab = maj if mode == 0 else mnr
    pos = tab.index(tonic % 12) if (tonic % 12) in tab else 0
    return f"{pos + 1}{'A' if mode == 0 else 'B'}"


def key_from_numerical(notation):
    """Key::from_numerical, result.rs:113-140 -> (mode, tonic) or None."""
    import re

    if len(notation.encode()) < 2:
        return None
    num_str, suffix = notation[:-1], notation[-1]
    if not re.fullmatch(r"\+?[0-9]+", num_str):  # u32::from_str
        return None
    num = int(num_str)
    if not 1 <= num <= 12:
        return None
    maj = [0, 7, 2, 9, 4, 11, 6, 1, 8, 3, 10, 5]
    mnr = [9, 4, 11, 6, 1, 8, 3, 10, 5, 0, 7, 2]
    if suffix == "A":
        return (0, maj[num - 1])
    if suffix == "B":
        return (1, mnr[num - 1])
    return None


def _tri(v):
    return None if v < 0 else bool(v)


def result_to_dict(r: SdspResult) -> dict:
    """AnalysisResult as a plain dict (serde field names, result.rs:186-263)."""
    beats = [r.beats[i] for i in range(r.n_beats)] if r.n_beats else []
    downs = [r.downbeats[i] for i in range(r.n_downbeats)] if r.n_downbeats else []
    bars = [r.bars[i] for i in range(r.n_bars)] if r.n_bars else []
    warns = [r.warnings[i].decode() for i in range(r.n_warnings)] if r.n_warnings else []
    flags = [FLAG_NAMES[i] for i in range(4) if r.flags & (1 << i)]
    d = {
        "bpm": r.bpm,
        "bpm_confidence": r.bpm_confidence,
        "key": {"Major" if r.key_mode == 0 else "Minor": r.key_tonic},
        "key_name": key_name(r.key_mode, r.key_tonic),
        "key_confidence": r.key_confidence,
        "key_clarity": r.key_clarity,
        "beat_grid": {"downbeats": downs, "beats": beats, "bars": bars},
        "grid_stability": r.grid_stability,
        "metadata": {
            "duration_seconds": r.duration_seconds,
            "sample_rate": r.sample_rate,
            "processing_time_ms": r.processing_time_ms,
            "algorithm_version": r.algorithm_version.decode(),
            "onset_method_consensus": r.onset_method_consensus,
            "methods_used": ["energy_flux", "chroma_extraction", "key_detection"],
            "flags": flags,
            "confidence_warnings": warns,
            "tempogram_multi_res_triggered": _tri(r.tempogram_multi_res_triggered),
            "tempogram_multi_res_used": _tri(r.tempogram_multi_res_used),
            "tempogram_percussive_triggered": _tri(r.tempogram_percussive_triggered),
            "tempogram_percussive_used": _tri(r.tempogram_percussive_used),
        },
    }
    if r.has_tempogram_candidates:
        d["metadata"]["tempogram_candidates"] = [
            {
                "bpm": r.tempogram_candidates[i].bpm,
                "score": r.tempogram_candidates[i].score,
                "fft_norm": r.tempogram_candidates[i].fft_norm,
                "autocorr_norm": r.tempogram_candidates[i].autocorr_norm,
                "selected": bool(r.tempogram_candidates[i].selected),
            }
            for i in range(r.n_tempogram_candidates)
        ]
    return d
