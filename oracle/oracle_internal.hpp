// oracle_internal.hpp — CPU restatement of stratum-dsp's default analyze_audio() path.
//
// TEST INFRASTRUCTURE ONLY.  This code is the parity checker for the HIP engine in
// stratum-dsp_amd/ and the "port" CPU baseline in bench.py.  Nothing in the product links
// or calls it; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do.
//
// Every function follows the reference file:line it cites (paths under /root/reference).
// Arithmetic is f32 in the reference's order (sequential folds, no FMA: -ffp-contract=off);
// transcendentals go through include/sdsp_libm.h and FFTs through include/sdsp_fft_spec.h.
// Parity pinning: see oracle/README.md (integration-test ranges + known-answer tests of the
// reference's own test-suite; the FFT/libm layers are pinned to numpy / correctly rounded
// double references because the reference's rustfft/libm rounding is itself unpinned).
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/sdsp_fft_spec.h"
#include "../include/sdsp_libm.h"
#include "../include/stratum_hip.h"

namespace orc {

constexpr float EPS = 1e-10f;  // `const EPSILON: f32 = 1e-10` (every module)

// AnalysisError propagated with `?`  (src/error.rs:7-22)
struct AErr {
    int code;
    std::string msg;
};
[[noreturn]] inline void fail(int code, const std::string& m) { throw AErr{code, m}; }

struct Cx {
    float re, im;
};

// Vec<Vec<f32>> spectrogram, flat row-major [frame][bin]
struct Spec {
    size_t frames = 0, bins = 0;
    std::vector<float> d;
    float* row(size_t t) { return d.data() + t * bins; }
    const float* row(size_t t) const { return d.data() + t * bins; }
    bool empty() const { return frames == 0; }
};

// ---------- FFT (sdsp_fft_spec.h) ----------
void fft_complex(std::vector<Cx>& x);                          // in place, forward
void rfft(const float* x, size_t n, std::vector<Cx>& out);    // out: n/2+1 bins
Spec compute_stft(const float* s, size_t n, size_t frame_size, size_t hop);  // extractor.rs:301

// ---------- BPM estimate types (src/features/period/mod.rs) ----------
struct BpmCandidate {
    float bpm, confidence;
};
struct BpmEstimate {
    float bpm, confidence;
    uint32_t method_agreement;
};
struct TempoCand {  // TempogramCandidateDebug, tempogram.rs:47-54
    float bpm, score, fft_norm, autocorr_norm;
    bool selected;
};

// ---------- preprocessing + onsets ----------
void normalize_peak(std::vector<float>& x, float headroom_db);
void normalize_rms(std::vector<float>& x, float target_lufs, float headroom_db);
void normalize_lufs(std::vector<float>& x, uint32_t sr, float target_lufs, float headroom_db);
void detect_and_trim(const std::vector<float>& x, uint32_t sr, float threshold_db, uint32_t min_ms,
                     size_t frame_size, size_t* trim_start, size_t* trim_end,
                     std::vector<std::pair<size_t, size_t>>* silence_map = nullptr);
std::vector<size_t> energy_flux_onsets(const float* s, size_t n, size_t frame, size_t hop, float thr_db);
std::vector<size_t> spectral_flux_onsets(const Spec& m, float pct);
std::vector<size_t> hfc_onsets(const Spec& m, uint32_t sr, float pct);
struct OnsetCand {
    size_t time_samples;
    float time_seconds, confidence;
    uint32_t voted_by;
};
void hpss_decompose(const Spec& m, size_t margin, Spec* H, Spec* P);  // hpss.rs:71-172
std::vector<size_t> hpss_onsets(const Spec& p, float pct);            // hpss.rs:290-372
std::vector<OnsetCand> vote_onsets(const std::vector<size_t> lists[4], const float w[4], uint32_t tol_ms,
                                   uint32_t sr);

// ---------- legacy BPM (period/mod.rs, autocorrelation.rs, comb_filter.rs, candidate_filter.rs) ----------
struct Guardrails {
    float preferred_min, preferred_max, soft_min, soft_max, mul_preferred, mul_soft, mul_extreme;
};
bool estimate_bpm_legacy(const std::vector<size_t>& onsets, uint32_t sr, size_t hop, float min_bpm,
                         float max_bpm, float res, const Guardrails* g, BpmEstimate* out);

// ---------- tempogram (novelty.rs, tempogram*.rs, multi_resolution.rs) ----------
struct BandCfg {
    bool enabled;
    float low_max_hz, mid_max_hz, high_max_hz, w_full, w_low, w_mid, w_high;
    bool seed_only;
    float support_threshold, consensus_bonus;
    bool enable_mel;
    size_t mel_n_mels;
    float mel_fmin_hz, mel_fmax_hz;
    size_t mel_max_filter_bins;
    float w_mel, nw_spectral, nw_energy, nw_hfc;
    size_t local_mean_window, smooth_window, superflux_k;
};
std::vector<float> combined_full_novelty(const Spec& m, uint32_t sr, const BandCfg& c);
void tempogram_impl(const Spec& m, uint32_t sr, uint32_t hop, float min_bpm, float max_bpm, float res,
                    const BandCfg* band, BpmEstimate* est, std::vector<TempoCand>* cands);
void multi_resolution(const std::vector<float>& samples, uint32_t sr, size_t frame_size, float min_bpm,
                      float max_bpm, float res, size_t top_k, float w512, float w256, float w1024,
                      float structural_discount, float dt512, float margin_threshold, bool human_prior,
                      const BandCfg* band, BpmEstimate* est, std::vector<TempoCand>* c512);

// ---------- beat grid (beat_tracking/) ----------
struct BeatDiag {            // which branches generate_beat_grid took (test probes)
    bool variable = false;   // detect_tempo_variations flagged a variable segment (mod.rs:152-154)
    bool refined = false;    // the Bayesian / per-segment HMM beats replaced the HMM beats (:205-219)
    uint32_t beats_per_bar = 4;
};
bool generate_beat_grid(float bpm, float conf, const std::vector<float>& onsets_s, uint32_t sr,
                        std::vector<float>* beats, std::vector<float>* downbeats, float* stability,
                        BeatDiag* diag = nullptr);

// ---------- key (chroma/, key/) ----------
void harmonic_mask_inplace(Spec& s, size_t margin, float power);
void hpcp_frames(const Spec& s, uint32_t sr, size_t fft_size, float sigma, size_t peaks, size_t harmonics,
                 float decay, float mag_power, std::vector<float>* chroma12, std::vector<float>* energies);
void smooth_chroma_inplace(std::vector<float>& ch, size_t frames, size_t window);
// opt-in chroma front-ends (o_chroma.cpp)
struct HpcpCfg {
    float sigma = 0.5f, tuning = 0.0f;
    size_t peaks = 24, harmonics = 4;
    float decay = 0.6f, mag_power = 0.5f;
    bool whitening = false;
    size_t whitening_bins = 31;
    bool bass_blend = false;
    float bass_fmin = 55.0f, bass_fmax = 300.0f, bass_weight = 0.35f;
};
float estimate_tuning(const Spec& s, uint32_t sr, size_t fft_size, float fmin_hz, float fmax_hz, size_t frame_step,
                      float peak_rel_threshold);
void chroma_frames(const Spec& s, uint32_t sr, size_t fft_size, bool soft, float sigma, float tuning,
                   std::vector<float>* chroma12, std::vector<float>* energies);
void hpcp_frames_x(const Spec& s, uint32_t sr, size_t fft_size, const HpcpCfg& c, std::vector<float>* chroma12,
                   std::vector<float>* energies);
bool log_freq_chroma(const Spec& s, uint32_t sr, size_t fft_size, std::vector<float>* chroma12,
                     std::vector<float>* energies);
void beat_sync_chroma(const Spec& s, uint32_t sr, size_t fft_size, size_t hop, const std::vector<float>& beats,
                      bool soft, float sigma, float tuning, std::vector<float>* chroma12, std::vector<float>* energies);
void smooth_time_inplace(Spec& s, size_t margin);
void key_hpss_mask_inplace(Spec& s, uint32_t sr, size_t fft_size, float fmin_hz, float fmax_hz, size_t frame_step,
                           size_t time_margin, size_t freq_margin, float mask_power);

struct KeyResult {
    int mode;
    uint32_t tonic;
    float confidence;
    float scores[24];
    int order[24];  // key index (mode*12+tonic) of scores[i]
};
void key_templates(float major[12][12], float minor[12][12], int template_set = 0);
KeyResult detect_key_weighted(const float* chroma, size_t frames, const float* weights,
                              const float maj[12][12], const float min[12][12]);
float key_clarity(const float* sorted_scores, int n);
void sharpen_chroma_inplace(float* ch12, float power);
struct ModeHeuristic {
    bool on = false;  // enable_key_mode_heuristic || enable_key_minor_harmonic_bonus
    float third_margin = 0.0f, flip_ratio = 0.0f, bonus_w = 0.0f;
    bool bonus = false;
};
KeyResult detect_key_weighted_mode_heuristic(const float* chroma, size_t frames, const float* weights,
                                             const float maj[12][12], const float min[12][12],
                                             const ModeHeuristic& mh);
KeyResult detect_key_ensemble(const float* chroma, size_t frames, const float* weights, float kk_weight,
                              float temperley_weight);
// detect_key_multi_scale; returns false when no segment qualified (the caller falls back)
bool detect_key_multi_scale(const float* chroma, size_t frames, const float* weights, const float maj[12][12],
                            const float min[12][12], const std::vector<size_t>& lengths, size_t hop, float min_clarity,
                            const std::vector<float>* scale_weights, const ModeHeuristic& mh, KeyResult* out,
                            int* used_segments);

// ---------- unit probes (o_*.cpp "unit probes" sections; tests/test_oracle_units_*.py) ----------
// Entry points at the granularity of the reference's own unit tests.  A probe returns a count /
// 0 on success or -(AnalysisError code) on error, with the message kept for
// sdsp_oracle_probe_error().
extern std::string g_probe_err;
// Study switches (tools/key_near_study.py; never set by the parity tests): g_block_energy folds
// each HPCP frame energy in 64-bin blocks the way the GPU's default key path does (k_mask_rp /
// k_hpcp_band) instead of the reference's one sequential sum; g_key_trace, when
// non-null, receives per detect_key_weighted call its 24 raw scores and, in segment voting, the
// segment's clarity after them.
extern int g_block_energy;
extern std::vector<float>* g_key_trace;
template <class F>
int64_t probe_call(F f) {
    try {
        return f();
    } catch (const AErr& e) {
        g_probe_err = e.msg;
        return -(int64_t)e.code;
    }
}
// Vec<Vec<f32>> from a flat row-major buffer; row_lens (nullable) lets a test pass a ragged
// spectrogram: the reference's validate loops reject frame lengths that differ from frame 0's
void spec_from_rows(const float* d, size_t frames, size_t bins, const uint64_t* row_lens, Spec* out);
std::vector<float> superflux_novelty(const Spec& m, size_t k);                    // novelty.rs:336-393
std::vector<float> energy_flux_novelty(const Spec& m);                            // novelty.rs:477-545
std::vector<float> hfc_novelty(const Spec& m, uint32_t sr);                       // novelty.rs:687-772
std::vector<float> spectral_flux_novelty(const Spec& m);                          // novelty.rs:222-334
std::vector<float> combined_novelty_params(const std::vector<float>& s, const std::vector<float>& e,
                                           const std::vector<float>& h, float ws, float we, float wh,
                                           size_t lmw, size_t smw);              // novelty.rs:874-932

// ---------- trace (test probes) ----------
struct Trace {
    size_t trim_start = 0, trim_end = 0;
    std::vector<size_t> energy_onsets, spectral_onsets, hfc_onsets, chosen_onsets;
    bool has_legacy = false;
    BpmEstimate legacy{0, 0, 0};
    bool has_tempogram = false;
    BpmEstimate base{0, 0, 0}, mr{0, 0, 0};
    bool ambiguous = false, used_mr = false, ran_mr = false;
    std::vector<TempoCand> base_cands;
    std::vector<float> novelty_full;
    std::vector<float> chroma;    // smoothed, frames*12
    std::vector<float> energies;  // per key frame
    std::vector<float> weights;
    bool weights_used = false;
    float tuning = 0.0f;
    int used_segments = 0;
    BeatDiag beat;
};

}  // namespace orc
