//! Raw bindings of libstratum_hip.so (include/stratum_hip.h).  Every struct is `#[repr(C)]` and
//! field-for-field identical to the C declaration (tests/test_rust_shim.py checks the order and
//! the types against the header).

#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_void};

pub const SDSP_OK: i32 = 0;
pub const SDSP_ERR_INVALID_INPUT: i32 = 1;
pub const SDSP_ERR_DECODING: i32 = 2;
pub const SDSP_ERR_PROCESSING: i32 = 3;
pub const SDSP_ERR_NOT_IMPLEMENTED: i32 = 4;
pub const SDSP_ERR_NUMERICAL: i32 = 5;

pub const SDSP_NORM_PEAK: i32 = 0;
pub const SDSP_NORM_RMS: i32 = 1;
pub const SDSP_NORM_LOUDNESS: i32 = 2;
pub const SDSP_TEMPLATES_KRUMHANSL_KESSLER: i32 = 0;
pub const SDSP_TEMPLATES_TEMPERLEY: i32 = 1;

pub const SDSP_FLAG_MULTIMODAL_BPM: u32 = 1 << 0;
pub const SDSP_FLAG_WEAK_TONALITY: u32 = 1 << 1;
pub const SDSP_FLAG_TEMPO_VARIATION: u32 = 1 << 2;
pub const SDSP_FLAG_ONSET_DETECTION_AMBIGUOUS: u32 = 1 << 3;

/// `sdsp_config`: AnalysisConfig (src/config.rs:8-592), bool -> u8, usize -> u64,
/// Option<T> -> has_x + x, Vec<T> -> pointer + length, enums -> i32.
#[repr(C)]
#[derive(Clone, Copy)]
pub struct sdsp_config {
    pub min_amplitude_db: f32,
    pub normalization: i32,
    pub enable_normalization: u8,
    pub enable_silence_trimming: u8,
    pub enable_onset_consensus: u8,
    pub onset_threshold_percentile: f32,
    pub onset_consensus_tolerance_ms: u32,
    pub onset_consensus_weights: [f32; 4],
    pub enable_hpss_onsets: u8,
    pub hpss_margin: u64,
    pub force_legacy_bpm: u8,
    pub enable_bpm_fusion: u8,
    pub enable_legacy_bpm_guardrails: u8,
    pub enable_tempogram_multi_resolution: u8,
    pub tempogram_multi_res_top_k: u64,
    pub tempogram_multi_res_w512: f32,
    pub tempogram_multi_res_w256: f32,
    pub tempogram_multi_res_w1024: f32,
    pub tempogram_multi_res_structural_discount: f32,
    pub tempogram_multi_res_double_time_512_factor: f32,
    pub tempogram_multi_res_margin_threshold: f32,
    pub tempogram_multi_res_use_human_prior: u8,
    pub enable_tempogram_percussive_fallback: u8,
    pub enable_tempogram_band_fusion: u8,
    pub tempogram_band_low_max_hz: f32,
    pub tempogram_band_mid_max_hz: f32,
    pub tempogram_band_high_max_hz: f32,
    pub tempogram_band_w_full: f32,
    pub tempogram_band_w_low: f32,
    pub tempogram_band_w_mid: f32,
    pub tempogram_band_w_high: f32,
    pub tempogram_band_seed_only: u8,
    pub tempogram_band_support_threshold: f32,
    pub tempogram_band_consensus_bonus: f32,
    pub tempogram_novelty_w_spectral: f32,
    pub tempogram_novelty_w_energy: f32,
    pub tempogram_novelty_w_hfc: f32,
    pub tempogram_novelty_local_mean_window: u64,
    pub tempogram_novelty_smooth_window: u64,
    pub has_debug_track_id: u8,
    pub debug_track_id: u32,
    pub has_debug_gt_bpm: u8,
    pub debug_gt_bpm: f32,
    pub debug_top_n: u64,
    pub enable_tempogram_mel_novelty: u8,
    pub tempogram_mel_n_mels: u64,
    pub tempogram_mel_fmin_hz: f32,
    pub tempogram_mel_fmax_hz: f32,
    pub tempogram_mel_max_filter_bins: u64,
    pub tempogram_mel_weight: f32,
    pub tempogram_superflux_max_filter_bins: u64,
    pub emit_tempogram_candidates: u8,
    pub tempogram_candidates_top_n: u64,
    pub legacy_bpm_preferred_min: f32,
    pub legacy_bpm_preferred_max: f32,
    pub legacy_bpm_soft_min: f32,
    pub legacy_bpm_soft_max: f32,
    pub legacy_bpm_conf_mul_preferred: f32,
    pub legacy_bpm_conf_mul_soft: f32,
    pub legacy_bpm_conf_mul_extreme: f32,
    pub min_bpm: f32,
    pub max_bpm: f32,
    pub bpm_resolution: f32,
    pub frame_size: u64,
    pub hop_size: u64,
    pub center_frequency: f32,
    pub soft_chroma_mapping: u8,
    pub soft_mapping_sigma: f32,
    pub chroma_sharpening_power: f32,
    pub enable_key_spectrogram_time_smoothing: u8,
    pub key_spectrogram_smooth_margin: u64,
    pub enable_key_frame_weighting: u8,
    pub key_min_tonalness: f32,
    pub key_tonalness_power: f32,
    pub key_energy_power: f32,
    pub enable_key_harmonic_mask: u8,
    pub key_harmonic_mask_power: f32,
    pub enable_key_hpss_harmonic: u8,
    pub key_hpss_frame_step: u64,
    pub key_hpss_time_margin: u64,
    pub key_hpss_freq_margin: u64,
    pub key_hpss_mask_power: f32,
    pub enable_key_stft_override: u8,
    pub key_stft_frame_size: u64,
    pub key_stft_hop_size: u64,
    pub enable_key_log_frequency: u8,
    pub enable_key_beat_synchronous: u8,
    pub enable_key_multi_scale: u8,
    pub key_template_set: i32,
    pub enable_key_ensemble: u8,
    pub key_ensemble_kk_weight: f32,
    pub key_ensemble_temperley_weight: f32,
    pub enable_key_median: u8,
    pub key_median_segment_length_frames: u64,
    pub key_median_segment_hop_frames: u64,
    pub key_median_min_segments: u64,
    pub key_multi_scale_lengths: *const u64,
    pub key_multi_scale_lengths_len: u64,
    pub key_multi_scale_hop: u64,
    pub key_multi_scale_min_clarity: f32,
    pub key_multi_scale_weights: *const f32,
    pub key_multi_scale_weights_len: u64,
    pub enable_key_tuning_compensation: u8,
    pub key_tuning_max_abs_semitones: f32,
    pub key_tuning_frame_step: u64,
    pub key_tuning_peak_rel_threshold: f32,
    pub enable_key_edge_trim: u8,
    pub key_edge_trim_fraction: f32,
    pub enable_key_segment_voting: u8,
    pub key_segment_len_frames: u64,
    pub key_segment_hop_frames: u64,
    pub key_segment_min_clarity: f32,
    pub enable_key_mode_heuristic: u8,
    pub key_mode_third_ratio_margin: f32,
    pub key_mode_flip_min_score_ratio: f32,
    pub enable_key_hpcp: u8,
    pub key_hpcp_peaks_per_frame: u64,
    pub key_hpcp_num_harmonics: u64,
    pub key_hpcp_harmonic_decay: f32,
    pub key_hpcp_mag_power: f32,
    pub enable_key_hpcp_whitening: u8,
    pub key_hpcp_whitening_smooth_bins: u64,
    pub enable_key_hpcp_bass_blend: u8,
    pub key_hpcp_bass_fmin_hz: f32,
    pub key_hpcp_bass_fmax_hz: f32,
    pub key_hpcp_bass_weight: f32,
    pub enable_key_minor_harmonic_bonus: u8,
    pub key_minor_leading_tone_bonus_weight: f32,
    pub enable_ml_refinement: u8,
}

/// `sdsp_tempo_candidate`: TempoCandidateDebug (src/analysis/result.rs:168-181)
#[repr(C)]
#[derive(Clone, Copy)]
pub struct sdsp_tempo_candidate {
    pub bpm: f32,
    pub score: f32,
    pub fft_norm: f32,
    pub autocorr_norm: f32,
    pub selected: u8,
}

/// `sdsp_result`: AnalysisResult + AnalysisMetadata + BeatGrid (src/analysis/result.rs:144-263);
/// the arrays are owned by the library until `sdsp_result_free`.
#[repr(C)]
pub struct sdsp_result {
    pub bpm: f32,
    pub bpm_confidence: f32,
    pub key_mode: i32,
    pub key_tonic: u32,
    pub key_confidence: f32,
    pub key_clarity: f32,
    pub beats: *mut f32,
    pub n_beats: u64,
    pub downbeats: *mut f32,
    pub n_downbeats: u64,
    pub bars: *mut f32,
    pub n_bars: u64,
    pub grid_stability: f32,
    pub duration_seconds: f32,
    pub sample_rate: u32,
    pub processing_time_ms: f32,
    pub algorithm_version: [c_char; 16],
    pub onset_method_consensus: f32,
    pub methods_used: u32,
    pub flags: u32,
    pub warnings: *mut *mut c_char,
    pub n_warnings: u64,
    pub tempogram_candidates: *mut sdsp_tempo_candidate,
    pub n_tempogram_candidates: u64,
    pub has_tempogram_candidates: i8,
    pub tempogram_multi_res_triggered: i8,
    pub tempogram_multi_res_used: i8,
    pub tempogram_percussive_triggered: i8,
    pub tempogram_percussive_used: i8,
    pub status: i32,
    pub error_message: [c_char; 256],
}

extern "C" {
    pub fn sdsp_config_default(cfg: *mut sdsp_config);
    pub fn sdsp_analyze_audio(
        samples: *const f32,
        n_samples: u64,
        sample_rate: u32,
        cfg: *const sdsp_config,
        out: *mut sdsp_result,
        err: *mut c_char,
        errlen: u64,
    ) -> i32;
    pub fn sdsp_analyze_batch(
        tracks: *const *const f32,
        lens: *const u64,
        n_tracks: u64,
        sample_rate: u32,
        cfg: *const sdsp_config,
        device_mask: u32,
        outs: *mut sdsp_result,
    ) -> i32;
    pub fn sdsp_result_free(r: *mut sdsp_result);
    pub fn sdsp_key_name(key_mode: i32, key_tonic: u32, buf: *mut c_char, buflen: u64) -> i32;
    pub fn sdsp_device_count() -> i32;
    pub fn sdsp_version() -> *const c_char;
    pub fn sdsp_analyze_batch_device(
        d_samples: *const f32,
        offsets: *const u64,
        lens: *const u64,
        n_tracks: u64,
        sample_rate: u32,
        cfg: *const sdsp_config,
        device: i32,
        stream: *mut c_void,
        outs: *mut sdsp_result,
    ) -> i32;
}
