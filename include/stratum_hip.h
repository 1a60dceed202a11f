/*
 * stratum_hip.h — C ABI of the MI355X-native analyze_audio() engine (libstratum_hip.so).
 *
 * This is the drop-in boundary for the reference crate's public API
 * (HLLMR/stratum-dsp, /root/reference):
 *
 *   pub fn analyze_audio(samples: &[f32], sample_rate: u32, config: AnalysisConfig)
 *       -> Result<AnalysisResult, AnalysisError>                      src/lib.rs:86-90
 *   impl Default for AnalysisConfig                                    src/config.rs:594-744
 *   pub struct AnalysisResult / AnalysisMetadata / BeatGrid / Key      src/analysis/result.rs:7-263
 *   pub enum AnalysisError (+ Display)                                 src/error.rs:7-34
 *
 * The Rust side binds these with `extern "C"` declarations (INTEGRATION.md shows the shim);
 * every struct here is `#[repr(C)]`-compatible: fixed-width scalars, pointer + length for
 * Vec fields, int32 for enums, int8 tri-states for Option<bool>.
 *
 * Ownership mirrors the reference: samples are borrowed (the library copies what it
 * needs, src/lib.rs:113), the config is read-only, results are owned by the library
 * until sdsp_result_free() is called.
 *
 * Threading: every entry point is reentrant.  Concurrent callers are serialised per
 * device inside the library (one HIP stream + workspace per device).
 */
#ifndef STRATUM_HIP_H
#define STRATUM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDSP_ABI_VERSION 1

/* AnalysisError variants, src/error.rs:7-22 (0 = Ok) */
enum sdsp_status {
    SDSP_OK = 0,
    SDSP_ERR_INVALID_INPUT = 1,    /* "Invalid input: {}"    */
    SDSP_ERR_DECODING = 2,         /* "Decoding error: {}"   */
    SDSP_ERR_PROCESSING = 3,       /* "Processing error: {}" */
    SDSP_ERR_NOT_IMPLEMENTED = 4,  /* "Not implemented: {}"  */
    SDSP_ERR_NUMERICAL = 5         /* "Numerical error: {}"  */
};

/* NormalizationMethod, src/preprocessing/normalization.rs:30-37 */
enum sdsp_normalization { SDSP_NORM_PEAK = 0, SDSP_NORM_RMS = 1, SDSP_NORM_LOUDNESS = 2 };
/* TemplateSet, src/features/key/templates.rs:17-22 */
enum sdsp_template_set { SDSP_TEMPLATES_KRUMHANSL_KESSLER = 0, SDSP_TEMPLATES_TEMPERLEY = 1 };

/*
 * AnalysisConfig, src/config.rs:8-592 — every pub field, same name, same meaning.
 * bool -> uint8_t, usize -> uint64_t, Option<T> -> has_x flag + value, Vec<T> -> ptr + len.
 */
typedef struct sdsp_config {
    float min_amplitude_db;
    int32_t normalization; /* enum sdsp_normalization */
    uint8_t enable_normalization;
    uint8_t enable_silence_trimming;
    uint8_t enable_onset_consensus;
    float onset_threshold_percentile;
    uint32_t onset_consensus_tolerance_ms;
    float onset_consensus_weights[4];
    uint8_t enable_hpss_onsets;
    uint64_t hpss_margin;
    uint8_t force_legacy_bpm;
    uint8_t enable_bpm_fusion;
    uint8_t enable_legacy_bpm_guardrails;
    uint8_t enable_tempogram_multi_resolution;
    uint64_t tempogram_multi_res_top_k;
    float tempogram_multi_res_w512;
    float tempogram_multi_res_w256;
    float tempogram_multi_res_w1024;
    float tempogram_multi_res_structural_discount;
    float tempogram_multi_res_double_time_512_factor;
    float tempogram_multi_res_margin_threshold;
    uint8_t tempogram_multi_res_use_human_prior;
    uint8_t enable_tempogram_percussive_fallback;
    uint8_t enable_tempogram_band_fusion;
    float tempogram_band_low_max_hz;
    float tempogram_band_mid_max_hz;
    float tempogram_band_high_max_hz;
    float tempogram_band_w_full;
    float tempogram_band_w_low;
    float tempogram_band_w_mid;
    float tempogram_band_w_high;
    uint8_t tempogram_band_seed_only;
    float tempogram_band_support_threshold;
    float tempogram_band_consensus_bonus;
    float tempogram_novelty_w_spectral;
    float tempogram_novelty_w_energy;
    float tempogram_novelty_w_hfc;
    uint64_t tempogram_novelty_local_mean_window;
    uint64_t tempogram_novelty_smooth_window;
    uint8_t has_debug_track_id;
    uint32_t debug_track_id;
    uint8_t has_debug_gt_bpm;
    float debug_gt_bpm;
    uint64_t debug_top_n;
    uint8_t enable_tempogram_mel_novelty;
    uint64_t tempogram_mel_n_mels;
    float tempogram_mel_fmin_hz;
    float tempogram_mel_fmax_hz;
    uint64_t tempogram_mel_max_filter_bins;
    float tempogram_mel_weight;
    uint64_t tempogram_superflux_max_filter_bins;
    uint8_t emit_tempogram_candidates;
    uint64_t tempogram_candidates_top_n;
    float legacy_bpm_preferred_min;
    float legacy_bpm_preferred_max;
    float legacy_bpm_soft_min;
    float legacy_bpm_soft_max;
    float legacy_bpm_conf_mul_preferred;
    float legacy_bpm_conf_mul_soft;
    float legacy_bpm_conf_mul_extreme;
    float min_bpm;
    float max_bpm;
    float bpm_resolution;
    uint64_t frame_size;
    uint64_t hop_size;
    float center_frequency;
    uint8_t soft_chroma_mapping;
    float soft_mapping_sigma;
    float chroma_sharpening_power;
    uint8_t enable_key_spectrogram_time_smoothing;
    uint64_t key_spectrogram_smooth_margin;
    uint8_t enable_key_frame_weighting;
    float key_min_tonalness;
    float key_tonalness_power;
    float key_energy_power;
    uint8_t enable_key_harmonic_mask;
    float key_harmonic_mask_power;
    uint8_t enable_key_hpss_harmonic;
    uint64_t key_hpss_frame_step;
    uint64_t key_hpss_time_margin;
    uint64_t key_hpss_freq_margin;
    float key_hpss_mask_power;
    uint8_t enable_key_stft_override;
    uint64_t key_stft_frame_size;
    uint64_t key_stft_hop_size;
    uint8_t enable_key_log_frequency;
    uint8_t enable_key_beat_synchronous;
    uint8_t enable_key_multi_scale;
    int32_t key_template_set; /* enum sdsp_template_set */
    uint8_t enable_key_ensemble;
    float key_ensemble_kk_weight;
    float key_ensemble_temperley_weight;
    uint8_t enable_key_median;
    uint64_t key_median_segment_length_frames;
    uint64_t key_median_segment_hop_frames;
    uint64_t key_median_min_segments;
    const uint64_t* key_multi_scale_lengths; /* Vec<usize> */
    uint64_t key_multi_scale_lengths_len;
    uint64_t key_multi_scale_hop;
    float key_multi_scale_min_clarity;
    const float* key_multi_scale_weights; /* Vec<f32> */
    uint64_t key_multi_scale_weights_len;
    uint8_t enable_key_tuning_compensation;
    float key_tuning_max_abs_semitones;
    uint64_t key_tuning_frame_step;
    float key_tuning_peak_rel_threshold;
    uint8_t enable_key_edge_trim;
    float key_edge_trim_fraction;
    uint8_t enable_key_segment_voting;
    uint64_t key_segment_len_frames;
    uint64_t key_segment_hop_frames;
    float key_segment_min_clarity;
    uint8_t enable_key_mode_heuristic;
    float key_mode_third_ratio_margin;
    float key_mode_flip_min_score_ratio;
    uint8_t enable_key_hpcp;
    uint64_t key_hpcp_peaks_per_frame;
    uint64_t key_hpcp_num_harmonics;
    float key_hpcp_harmonic_decay;
    float key_hpcp_mag_power;
    uint8_t enable_key_hpcp_whitening;
    uint64_t key_hpcp_whitening_smooth_bins;
    uint8_t enable_key_hpcp_bass_blend;
    float key_hpcp_bass_fmin_hz;
    float key_hpcp_bass_fmax_hz;
    float key_hpcp_bass_weight;
    uint8_t enable_key_minor_harmonic_bonus;
    float key_minor_leading_tone_bonus_weight;
    uint8_t enable_ml_refinement; /* #[cfg(feature = "ml")] */
} sdsp_config;

/* AnalysisFlag, src/analysis/result.rs:157-166 — bit i set <=> flags contains variant i */
enum sdsp_flag {
    SDSP_FLAG_MULTIMODAL_BPM = 1u << 0,
    SDSP_FLAG_WEAK_TONALITY = 1u << 1,
    SDSP_FLAG_TEMPO_VARIATION = 1u << 2,
    SDSP_FLAG_ONSET_DETECTION_AMBIGUOUS = 1u << 3
};

/* TempoCandidateDebug, src/analysis/result.rs:168-181 */
typedef struct sdsp_tempo_candidate {
    float bpm;
    float score;
    float fft_norm;
    float autocorr_norm;
    uint8_t selected;
} sdsp_tempo_candidate;

/* Key, src/analysis/result.rs:7-12 */
enum sdsp_key_mode { SDSP_KEY_MAJOR = 0, SDSP_KEY_MINOR = 1 };

/* AnalysisResult + AnalysisMetadata + BeatGrid, src/analysis/result.rs:144-263 */
typedef struct sdsp_result {
    float bpm;
    float bpm_confidence;
    int32_t key_mode;   /* enum sdsp_key_mode */
    uint32_t key_tonic; /* 0 = C .. 11 = B */
    float key_confidence;
    float key_clarity;
    /* beat_grid (library-owned arrays) */
    float* beats;
    uint64_t n_beats;
    float* downbeats;
    uint64_t n_downbeats;
    float* bars;
    uint64_t n_bars;
    float grid_stability;
    /* metadata */
    float duration_seconds;
    uint32_t sample_rate;
    float processing_time_ms;
    char algorithm_version[16];
    float onset_method_consensus;
    uint32_t methods_used; /* always energy_flux|chroma_extraction|key_detection (lib.rs:1606-1610) */
    uint32_t flags;        /* enum sdsp_flag bitmask, in reference push order */
    char** warnings;       /* confidence_warnings, in order */
    uint64_t n_warnings;
    sdsp_tempo_candidate* tempogram_candidates; /* valid iff has_tempogram_candidates */
    uint64_t n_tempogram_candidates;
    int8_t has_tempogram_candidates;
    /* Option<bool>: -1 = None, 0 = Some(false), 1 = Some(true) */
    int8_t tempogram_multi_res_triggered;
    int8_t tempogram_multi_res_used;
    int8_t tempogram_percussive_triggered;
    int8_t tempogram_percussive_used;
    /* per-track status for the batch entry points (enum sdsp_status + Display text) */
    int32_t status;
    char error_message[256];
} sdsp_result;

/* AnalysisConfig::default(), src/config.rs:594-744 */
void sdsp_config_default(sdsp_config* cfg);

/*
 * analyze_audio(samples, sample_rate, config), src/lib.rs:86.
 * Returns enum sdsp_status; on error the Display text ("Invalid input: Empty audio samples")
 * is written to err (NUL-terminated, truncated to errlen) and *out is left zeroed.
 */
int32_t sdsp_analyze_audio(const float* samples, uint64_t n_samples, uint32_t sample_rate,
                           const sdsp_config* cfg, sdsp_result* out, char* err, uint64_t errlen);

/*
 * Batch form (new): N independent analyze_audio calls, sharded over the devices in
 * device_mask (bit d = HIP device d; 0 = device 0).  outs[i].status carries each track's
 * Ok/Err.  Returns SDSP_OK unless the batch itself could not run.
 */
int32_t sdsp_analyze_batch(const float* const* tracks, const uint64_t* lens, uint64_t n_tracks,
                           uint32_t sample_rate, const sdsp_config* cfg, uint32_t device_mask,
                           sdsp_result* outs);

/*
 * Device-resident batch: tracks already in HBM on `device` (concatenated, track i starts at
 * d_samples + offsets[i] and has lens[i] samples; host arrays).  `stream` is a hipStream_t
 * (NULL = the library's own stream).  Used by the throughput benchmark.
 */
int32_t sdsp_analyze_batch_device(const float* d_samples, const uint64_t* offsets,
                                  const uint64_t* lens, uint64_t n_tracks, uint32_t sample_rate,
                                  const sdsp_config* cfg, int32_t device, void* stream,
                                  sdsp_result* outs);

/*
 * Stage selection for the device-resident batch (new; the reference has no such switch).
 * SDSP_STAGES_BPM_ONLY runs the tempo path alone -- src/lib.rs:86-910, SURVEY.md rows a1-a19:
 * normalisation, trim, onsets, tempogram, multi-resolution escalation, BPM choice.  bpm,
 * bpm_confidence, duration and the tempogram_* flags equal a full run's; the key fields keep their
 * defaults (C major, 0) and the beat grid is empty.  BASELINE config 5 is quoted in this mode.
 */
enum sdsp_stages { SDSP_STAGES_FULL = 0, SDSP_STAGES_BPM_ONLY = 1 };
int32_t sdsp_analyze_batch_device_ex(const float* d_samples, const uint64_t* offsets,
                                     const uint64_t* lens, uint64_t n_tracks, uint32_t sample_rate,
                                     const sdsp_config* cfg, int32_t device, void* stream,
                                     int32_t stages, sdsp_result* outs);

/* Frees the arrays owned by one result (beats, downbeats, bars, warnings, candidates). */
void sdsp_result_free(sdsp_result* r);

/*
 * Synthetic track generator on device: writes n_tracks tracks of `len`
 * samples each, track i at d_out + i*len, seeds seed0 + i.  bpm_out/key_out (host, may be
 * NULL) receive the generated tempo and key (key = mode*12 + tonic).  bpm_mode 0 = uniform
 * [70,180] on a 0.5 grid; 1 = thirds in [55,80], [170,200], [80,170] (config 5).
 */
int32_t sdsp_generate_synthetic(float* d_out, uint64_t n_tracks, uint64_t len, uint32_t sample_rate,
                                uint64_t seed0, int32_t bpm_mode, int32_t device, void* stream,
                                float* bpm_out, int32_t* key_out);

/*
 * Device-memory plumbing for harnesses that hold tracks in HBM (benchmarks, tests).  The engine
 * links the system ROCm HIP runtime; callers that use these need no second GPU runtime.
 */
int32_t sdsp_device_count(void);
int32_t sdsp_device_malloc(int32_t device, uint64_t bytes, void** ptr);
int32_t sdsp_device_free(int32_t device, void* ptr);
int32_t sdsp_memcpy_h2d(int32_t device, void* dst, const void* src, uint64_t bytes);
int32_t sdsp_memcpy_d2h(int32_t device, void* dst, const void* src, uint64_t bytes);
int32_t sdsp_device_synchronize(int32_t device);

/*
 * compute_confidence (src/analysis/confidence.rs:121-297): host-side scores of one result.
 * flag_list holds AnalysisFlag indices (0 MultimodalBpm, 1 WeakTonality, 2 TempoVariation,
 * 3 OnsetDetectionAmbiguous) in the reference's push order, duplicates kept (the result's own
 * flags first, then MultimodalBpm / WeakTonality / TempoVariation as their thresholds fire).
 */
typedef struct sdsp_confidence {
    float bpm_confidence;
    float key_confidence;
    float grid_stability;
    float overall_confidence;
    uint32_t n_flags;
    int32_t flag_list[8];
} sdsp_confidence;
int32_t sdsp_compute_confidence(const sdsp_result* result, sdsp_confidence* out);

/* Key::name (src/analysis/result.rs:31-39): "C", "F#", "Am", "C#m"; returns the length. */
int32_t sdsp_key_name(int32_t key_mode, uint32_t key_tonic, char* buf, uint64_t buflen);

/*
 * Audio decode front-end (examples/analyze_file.rs:25-180, analyze_batch.rs:30-177), by magic
 * number: RIFF/WAVE (PCM u8 / s16 / s24 / s32, IEEE float f32 / f64, G.711, IMA and Microsoft
 * ADPCM, WAVE_FORMAT_EXTENSIBLE with those sub-formats), AIFF / AIFF-C, CAF (lpcm, G.711, ALAC),
 * FLAC (native or in Ogg; 8-32 bits, 1-8 channels; symphonia's S32 buffers, sample << (32 -
 * bps)), ALAC in ISO MP4 / M4A, Ogg Vorbis, and Matroska / WebM carrying PCM, FLAC, ALAC or
 * Vorbis -- decoded to mono f32 as the reference's
 * symphonia path converts its buffers (s16 / 32768, s24 / 8388608, s32 / 2147483648, (u8 - 128) /
 * 128, f64 -> f32, f32 as is; channels summed in order and divided by the channel count).  A
 * packet that fails to decode (a FLAC frame failing its CRC, a damaged ALAC packet, an Ogg page
 * failing its CRC) is skipped, as the examples skip such a packet.  *samples is malloc'ed (free
 * with sdsp_free_samples).  Returns 0, or SDSP_ERR_DECODING with the reason in err (MP3 / MP2 /
 * MP1, AAC and Opus are named as unsupported codecs).
 */
int32_t sdsp_decode_audio_file(const char* path, float** samples, uint64_t* n_samples, uint32_t* sample_rate,
                               char* err, uint64_t errlen);
void sdsp_free_samples(float* samples);

/* Library identification: "stratum-hip <abi> gfx950" */
const char* sdsp_version(void);

/* Per-kernel timing of the last batch on `device` (bench/roofline), milliseconds. */
typedef struct sdsp_stage_times {
    double stft2048_ms;     /* k_stft_mag<2048> launches, summed */
    double stft8192_ms;     /* k_stft_mag<8192> launches, summed */
    double features_ms;     /* frame features + novelty */
    double tempogram_ms;    /* FFT + autocorrelation tempograms + candidate scoring */
    double key_ms;          /* mask + HPCP + key voting */
    double beat_ms;         /* onset consensus + beat grid */
    double total_ms;        /* whole batch, device time */
    uint64_t stft2048_launches;
    uint64_t stft8192_launches;
    double stft2048_bytes;  /* algorithmic bytes: 4*N_in + 4*F*(nfft/2+1) per STFT */
    double stft8192_bytes;
    uint64_t stft2048_frames; /* frames the STFT launches computed (the VALU census is per frame) */
    uint64_t stft8192_frames;
    uint64_t key_reruns;      /* tracks analysed again with the sequential key-energy fold (near a
                                 key decision under the block-folded energies) */
    double rerun_ms;          /* wall time of that rerun (included in total_ms) */
} sdsp_stage_times;
int32_t sdsp_last_stage_times(int32_t device, sdsp_stage_times* out);

#ifdef __cplusplus
}
#endif

#endif /* STRATUM_HIP_H */
