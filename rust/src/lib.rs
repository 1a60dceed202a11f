//! stratum-dsp-hip: the reference crate's `analyze_audio` hot path on MI355X.
//!
//! A drop-in for `stratum_dsp::analyze_audio` (/root/reference/src/lib.rs:86-90): same
//! signature, same `AnalysisConfig` / `AnalysisResult` / `AnalysisError` types (taken from the
//! reference crate itself), computed by libstratum_hip.so through the C ABI of
//! include/stratum_hip.h.  A caller switches with one `use` line:
//!
//! ```ignore
//! // use stratum_dsp::analyze_audio;
//! use stratum_dsp_hip::analyze_audio;
//! let result = analyze_audio(&samples, 44_100, AnalysisConfig::default())?;
//! ```
//!
//! `analyze_batch` is the throughput form (many tracks per call, sharded over the GPUs of
//! `device_mask`) that replaces the caller-side rayon fan-out of
//! /root/reference/examples/analyze_batch.rs:239-268.
//!
//! Not compiled in this repository's build (the image has no Rust toolchain); INTEGRATION.md
//! gives the build recipe.  tests/test_rust_shim.py checks the field mapping against the header.

pub mod ffi;

use std::ffi::CStr;
use std::os::raw::c_char;

use stratum_dsp::analysis::result::{AnalysisFlag, TempoCandidateDebug};
use stratum_dsp::features::key::templates::TemplateSet;
use stratum_dsp::preprocessing::normalization::NormalizationMethod;
use stratum_dsp::{AnalysisConfig, AnalysisError, AnalysisMetadata, AnalysisResult, BeatGrid, Key};

/// Host storage an `sdsp_config` points into, kept alive for the duration of the call.
struct Keep {
    multi_scale_lengths: Vec<u64>, // Vec<usize> -> u64 (usize is 64-bit on every ROCm host)
}

fn normalization_to_c(m: &NormalizationMethod) -> i32 {
    match m {
        NormalizationMethod::Peak => ffi::SDSP_NORM_PEAK,
        NormalizationMethod::RMS => ffi::SDSP_NORM_RMS,
        NormalizationMethod::Loudness => ffi::SDSP_NORM_LOUDNESS,
    }
}

fn template_set_to_c(t: &TemplateSet) -> i32 {
    match t {
        TemplateSet::KrumhanslKessler => ffi::SDSP_TEMPLATES_KRUMHANSL_KESSLER,
        TemplateSet::Temperley => ffi::SDSP_TEMPLATES_TEMPERLEY,
    }
}

#[cfg(feature = "ml")]
fn ml_refinement(c: &AnalysisConfig) -> u8 {
    c.enable_ml_refinement as u8 // the engine answers NotImplemented (no model ships)
}
#[cfg(not(feature = "ml"))]
fn ml_refinement(_c: &AnalysisConfig) -> u8 {
    0
}

/// AnalysisConfig (src/config.rs:8-592) -> sdsp_config, every pub field by name.  The returned
/// `Keep` owns the converted `key_multi_scale_lengths`; `key_multi_scale_weights` points into `c`.
fn to_c(c: &AnalysisConfig) -> (ffi::sdsp_config, Keep) {
    let keep = Keep {
        multi_scale_lengths: c.key_multi_scale_lengths.iter().map(|&v| v as u64).collect(),
    };
    let cfg = ffi::sdsp_config {
        min_amplitude_db: c.min_amplitude_db,
        normalization: normalization_to_c(&c.normalization),
        enable_normalization: c.enable_normalization as u8,
        enable_silence_trimming: c.enable_silence_trimming as u8,
        enable_onset_consensus: c.enable_onset_consensus as u8,
        onset_threshold_percentile: c.onset_threshold_percentile,
        onset_consensus_tolerance_ms: c.onset_consensus_tolerance_ms,
        onset_consensus_weights: c.onset_consensus_weights,
        enable_hpss_onsets: c.enable_hpss_onsets as u8,
        hpss_margin: c.hpss_margin as u64,
        force_legacy_bpm: c.force_legacy_bpm as u8,
        enable_bpm_fusion: c.enable_bpm_fusion as u8,
        enable_legacy_bpm_guardrails: c.enable_legacy_bpm_guardrails as u8,
        enable_tempogram_multi_resolution: c.enable_tempogram_multi_resolution as u8,
        tempogram_multi_res_top_k: c.tempogram_multi_res_top_k as u64,
        tempogram_multi_res_w512: c.tempogram_multi_res_w512,
        tempogram_multi_res_w256: c.tempogram_multi_res_w256,
        tempogram_multi_res_w1024: c.tempogram_multi_res_w1024,
        tempogram_multi_res_structural_discount: c.tempogram_multi_res_structural_discount,
        tempogram_multi_res_double_time_512_factor: c.tempogram_multi_res_double_time_512_factor,
        tempogram_multi_res_margin_threshold: c.tempogram_multi_res_margin_threshold,
        tempogram_multi_res_use_human_prior: c.tempogram_multi_res_use_human_prior as u8,
        enable_tempogram_percussive_fallback: c.enable_tempogram_percussive_fallback as u8,
        enable_tempogram_band_fusion: c.enable_tempogram_band_fusion as u8,
        tempogram_band_low_max_hz: c.tempogram_band_low_max_hz,
        tempogram_band_mid_max_hz: c.tempogram_band_mid_max_hz,
        tempogram_band_high_max_hz: c.tempogram_band_high_max_hz,
        tempogram_band_w_full: c.tempogram_band_w_full,
        tempogram_band_w_low: c.tempogram_band_w_low,
        tempogram_band_w_mid: c.tempogram_band_w_mid,
        tempogram_band_w_high: c.tempogram_band_w_high,
        tempogram_band_seed_only: c.tempogram_band_seed_only as u8,
        tempogram_band_support_threshold: c.tempogram_band_support_threshold,
        tempogram_band_consensus_bonus: c.tempogram_band_consensus_bonus,
        tempogram_novelty_w_spectral: c.tempogram_novelty_w_spectral,
        tempogram_novelty_w_energy: c.tempogram_novelty_w_energy,
        tempogram_novelty_w_hfc: c.tempogram_novelty_w_hfc,
        tempogram_novelty_local_mean_window: c.tempogram_novelty_local_mean_window as u64,
        tempogram_novelty_smooth_window: c.tempogram_novelty_smooth_window as u64,
        has_debug_track_id: c.debug_track_id.is_some() as u8,
        debug_track_id: c.debug_track_id.unwrap_or(0),
        has_debug_gt_bpm: c.debug_gt_bpm.is_some() as u8,
        debug_gt_bpm: c.debug_gt_bpm.unwrap_or(0.0),
        debug_top_n: c.debug_top_n as u64,
        enable_tempogram_mel_novelty: c.enable_tempogram_mel_novelty as u8,
        tempogram_mel_n_mels: c.tempogram_mel_n_mels as u64,
        tempogram_mel_fmin_hz: c.tempogram_mel_fmin_hz,
        tempogram_mel_fmax_hz: c.tempogram_mel_fmax_hz,
        tempogram_mel_max_filter_bins: c.tempogram_mel_max_filter_bins as u64,
        tempogram_mel_weight: c.tempogram_mel_weight,
        tempogram_superflux_max_filter_bins: c.tempogram_superflux_max_filter_bins as u64,
        emit_tempogram_candidates: c.emit_tempogram_candidates as u8,
        tempogram_candidates_top_n: c.tempogram_candidates_top_n as u64,
        legacy_bpm_preferred_min: c.legacy_bpm_preferred_min,
        legacy_bpm_preferred_max: c.legacy_bpm_preferred_max,
        legacy_bpm_soft_min: c.legacy_bpm_soft_min,
        legacy_bpm_soft_max: c.legacy_bpm_soft_max,
        legacy_bpm_conf_mul_preferred: c.legacy_bpm_conf_mul_preferred,
        legacy_bpm_conf_mul_soft: c.legacy_bpm_conf_mul_soft,
        legacy_bpm_conf_mul_extreme: c.legacy_bpm_conf_mul_extreme,
        min_bpm: c.min_bpm,
        max_bpm: c.max_bpm,
        bpm_resolution: c.bpm_resolution,
        frame_size: c.frame_size as u64,
        hop_size: c.hop_size as u64,
        center_frequency: c.center_frequency,
        soft_chroma_mapping: c.soft_chroma_mapping as u8,
        soft_mapping_sigma: c.soft_mapping_sigma,
        chroma_sharpening_power: c.chroma_sharpening_power,
        enable_key_spectrogram_time_smoothing: c.enable_key_spectrogram_time_smoothing as u8,
        key_spectrogram_smooth_margin: c.key_spectrogram_smooth_margin as u64,
        enable_key_frame_weighting: c.enable_key_frame_weighting as u8,
        key_min_tonalness: c.key_min_tonalness,
        key_tonalness_power: c.key_tonalness_power,
        key_energy_power: c.key_energy_power,
        enable_key_harmonic_mask: c.enable_key_harmonic_mask as u8,
        key_harmonic_mask_power: c.key_harmonic_mask_power,
        enable_key_hpss_harmonic: c.enable_key_hpss_harmonic as u8,
        key_hpss_frame_step: c.key_hpss_frame_step as u64,
        key_hpss_time_margin: c.key_hpss_time_margin as u64,
        key_hpss_freq_margin: c.key_hpss_freq_margin as u64,
        key_hpss_mask_power: c.key_hpss_mask_power,
        enable_key_stft_override: c.enable_key_stft_override as u8,
        key_stft_frame_size: c.key_stft_frame_size as u64,
        key_stft_hop_size: c.key_stft_hop_size as u64,
        enable_key_log_frequency: c.enable_key_log_frequency as u8,
        enable_key_beat_synchronous: c.enable_key_beat_synchronous as u8,
        enable_key_multi_scale: c.enable_key_multi_scale as u8,
        key_template_set: template_set_to_c(&c.key_template_set),
        enable_key_ensemble: c.enable_key_ensemble as u8,
        key_ensemble_kk_weight: c.key_ensemble_kk_weight,
        key_ensemble_temperley_weight: c.key_ensemble_temperley_weight,
        enable_key_median: c.enable_key_median as u8,
        key_median_segment_length_frames: c.key_median_segment_length_frames as u64,
        key_median_segment_hop_frames: c.key_median_segment_hop_frames as u64,
        key_median_min_segments: c.key_median_min_segments as u64,
        key_multi_scale_lengths: keep.multi_scale_lengths.as_ptr(),
        key_multi_scale_lengths_len: c.key_multi_scale_lengths.len() as u64,
        key_multi_scale_hop: c.key_multi_scale_hop as u64,
        key_multi_scale_min_clarity: c.key_multi_scale_min_clarity,
        key_multi_scale_weights: c.key_multi_scale_weights.as_ptr(),
        key_multi_scale_weights_len: c.key_multi_scale_weights.len() as u64,
        enable_key_tuning_compensation: c.enable_key_tuning_compensation as u8,
        key_tuning_max_abs_semitones: c.key_tuning_max_abs_semitones,
        key_tuning_frame_step: c.key_tuning_frame_step as u64,
        key_tuning_peak_rel_threshold: c.key_tuning_peak_rel_threshold,
        enable_key_edge_trim: c.enable_key_edge_trim as u8,
        key_edge_trim_fraction: c.key_edge_trim_fraction,
        enable_key_segment_voting: c.enable_key_segment_voting as u8,
        key_segment_len_frames: c.key_segment_len_frames as u64,
        key_segment_hop_frames: c.key_segment_hop_frames as u64,
        key_segment_min_clarity: c.key_segment_min_clarity,
        enable_key_mode_heuristic: c.enable_key_mode_heuristic as u8,
        key_mode_third_ratio_margin: c.key_mode_third_ratio_margin,
        key_mode_flip_min_score_ratio: c.key_mode_flip_min_score_ratio,
        enable_key_hpcp: c.enable_key_hpcp as u8,
        key_hpcp_peaks_per_frame: c.key_hpcp_peaks_per_frame as u64,
        key_hpcp_num_harmonics: c.key_hpcp_num_harmonics as u64,
        key_hpcp_harmonic_decay: c.key_hpcp_harmonic_decay,
        key_hpcp_mag_power: c.key_hpcp_mag_power,
        enable_key_hpcp_whitening: c.enable_key_hpcp_whitening as u8,
        key_hpcp_whitening_smooth_bins: c.key_hpcp_whitening_smooth_bins as u64,
        enable_key_hpcp_bass_blend: c.enable_key_hpcp_bass_blend as u8,
        key_hpcp_bass_fmin_hz: c.key_hpcp_bass_fmin_hz,
        key_hpcp_bass_fmax_hz: c.key_hpcp_bass_fmax_hz,
        key_hpcp_bass_weight: c.key_hpcp_bass_weight,
        enable_key_minor_harmonic_bonus: c.enable_key_minor_harmonic_bonus as u8,
        key_minor_leading_tone_bonus_weight: c.key_minor_leading_tone_bonus_weight,
        enable_ml_refinement: ml_refinement(c),
    };
    (cfg, keep)
}

/// AnalysisError (src/error.rs:7-22) from a status code and the engine's Display text
/// ("Invalid input: ..."), whose variant prefix (src/error.rs:24-34) is stripped back off.
fn error_from_c(status: i32, text: &str) -> AnalysisError {
    let strip = |p: &str| text.strip_prefix(p).unwrap_or(text).to_string();
    match status {
        ffi::SDSP_ERR_INVALID_INPUT => AnalysisError::InvalidInput(strip("Invalid input: ")),
        ffi::SDSP_ERR_DECODING => AnalysisError::DecodingError(strip("Decoding error: ")),
        ffi::SDSP_ERR_NOT_IMPLEMENTED => AnalysisError::NotImplemented(strip("Not implemented: ")),
        ffi::SDSP_ERR_NUMERICAL => AnalysisError::NumericalError(strip("Numerical error: ")),
        _ => AnalysisError::ProcessingError(strip("Processing error: ")),
    }
}

fn c_str(p: *const c_char) -> String {
    if p.is_null() {
        return String::new();
    }
    unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
}

unsafe fn vec_of(p: *const f32, n: u64) -> Vec<f32> {
    if p.is_null() || n == 0 {
        Vec::new()
    } else {
        std::slice::from_raw_parts(p, n as usize).to_vec()
    }
}

fn tri(v: i8) -> Option<bool> {
    match v {
        0 => Some(false),
        1 => Some(true),
        _ => None,
    }
}

/// sdsp_result -> AnalysisResult (src/analysis/result.rs:144-263); copies every array, so the
/// caller frees `r` right after.
unsafe fn from_c(r: &ffi::sdsp_result) -> AnalysisResult {
    let key = if r.key_mode == 1 { Key::Minor(r.key_tonic) } else { Key::Major(r.key_tonic) };
    let mut flags = Vec::new();
    for (bit, f) in [
        (ffi::SDSP_FLAG_MULTIMODAL_BPM, AnalysisFlag::MultimodalBpm),
        (ffi::SDSP_FLAG_WEAK_TONALITY, AnalysisFlag::WeakTonality),
        (ffi::SDSP_FLAG_TEMPO_VARIATION, AnalysisFlag::TempoVariation),
        (ffi::SDSP_FLAG_ONSET_DETECTION_AMBIGUOUS, AnalysisFlag::OnsetDetectionAmbiguous),
    ] {
        if r.flags & bit != 0 {
            flags.push(f);
        }
    }
    let warnings = (0..r.n_warnings as usize).map(|i| c_str(*r.warnings.add(i))).collect();
    let tempogram_candidates = if r.has_tempogram_candidates != 0 {
        let n = r.n_tempogram_candidates as usize;
        Some(
            (0..n)
                .map(|i| {
                    let c = &*r.tempogram_candidates.add(i);
                    TempoCandidateDebug {
                        bpm: c.bpm,
                        score: c.score,
                        fft_norm: c.fft_norm,
                        autocorr_norm: c.autocorr_norm,
                        selected: c.selected != 0,
                    }
                })
                .collect(),
        )
    } else {
        None
    };
    AnalysisResult {
        bpm: r.bpm,
        bpm_confidence: r.bpm_confidence,
        key,
        key_confidence: r.key_confidence,
        key_clarity: r.key_clarity,
        beat_grid: BeatGrid {
            downbeats: vec_of(r.downbeats, r.n_downbeats),
            beats: vec_of(r.beats, r.n_beats),
            bars: vec_of(r.bars, r.n_bars),
        },
        grid_stability: r.grid_stability,
        metadata: AnalysisMetadata {
            duration_seconds: r.duration_seconds,
            sample_rate: r.sample_rate,
            processing_time_ms: r.processing_time_ms,
            algorithm_version: c_str(r.algorithm_version.as_ptr()),
            onset_method_consensus: r.onset_method_consensus,
            // src/lib.rs:1606-1610: always these three, in this order
            methods_used: vec!["energy_flux".into(), "chroma_extraction".into(), "key_detection".into()],
            flags,
            confidence_warnings: warnings,
            tempogram_candidates,
            tempogram_multi_res_triggered: tri(r.tempogram_multi_res_triggered),
            tempogram_multi_res_used: tri(r.tempogram_multi_res_used),
            tempogram_percussive_triggered: tri(r.tempogram_percussive_triggered),
            tempogram_percussive_used: tri(r.tempogram_percussive_used),
        },
    }
}

/// `stratum_dsp::analyze_audio` (src/lib.rs:86-1635) on the GPU: same inputs, same result type,
/// same error variants and messages.  The samples are borrowed; the engine copies them to HBM.
pub fn analyze_audio(
    samples: &[f32],
    sample_rate: u32,
    config: AnalysisConfig,
) -> Result<AnalysisResult, AnalysisError> {
    let (cfg, _keep) = to_c(&config);
    let mut out: ffi::sdsp_result = unsafe { std::mem::zeroed() };
    let mut err = [0 as c_char; 512];
    let st = unsafe {
        ffi::sdsp_analyze_audio(
            samples.as_ptr(),
            samples.len() as u64,
            sample_rate,
            &cfg,
            &mut out,
            err.as_mut_ptr(),
            err.len() as u64,
        )
    };
    if st != ffi::SDSP_OK {
        return Err(error_from_c(st, &c_str(err.as_ptr())));
    }
    let r = unsafe { from_c(&out) };
    unsafe { ffi::sdsp_result_free(&mut out) };
    Ok(r)
}

/// Many `analyze_audio` calls in one: track i of `tracks`, all at `sample_rate`, sharded over
/// the devices in `device_mask` (bit d = HIP device d; 0 = device 0).  Each track gets its own
/// Ok / Err, exactly as the per-track call would return it.
pub fn analyze_batch(
    tracks: &[&[f32]],
    sample_rate: u32,
    config: &AnalysisConfig,
    device_mask: u32,
) -> Result<Vec<Result<AnalysisResult, AnalysisError>>, AnalysisError> {
    let (cfg, _keep) = to_c(config);
    let ptrs: Vec<*const f32> = tracks.iter().map(|t| t.as_ptr()).collect();
    let lens: Vec<u64> = tracks.iter().map(|t| t.len() as u64).collect();
    let mut outs: Vec<ffi::sdsp_result> = (0..tracks.len()).map(|_| unsafe { std::mem::zeroed() }).collect();
    let st = unsafe {
        ffi::sdsp_analyze_batch(
            ptrs.as_ptr(),
            lens.as_ptr(),
            tracks.len() as u64,
            sample_rate,
            &cfg,
            device_mask,
            outs.as_mut_ptr(),
        )
    };
    let results = outs
        .iter_mut()
        .map(|o| {
            let r = if o.status == ffi::SDSP_OK {
                Ok(unsafe { from_c(o) })
            } else {
                Err(error_from_c(o.status, &c_str(o.error_message.as_ptr())))
            };
            unsafe { ffi::sdsp_result_free(o) };
            r
        })
        .collect();
    if st != ffi::SDSP_OK {
        // a chunk or device failed as a whole: its tracks already carry that error
        log_batch_failure(st);
    }
    Ok(results)
}

fn log_batch_failure(st: i32) {
    eprintln!("stratum-dsp-hip: analyze_batch returned status {st}; per-track statuses hold the details");
}

/// The library's identification string ("stratum-hip <abi> gfx950").
pub fn version() -> String {
    c_str(unsafe { ffi::sdsp_version() })
}
