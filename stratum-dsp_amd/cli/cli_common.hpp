// cli_common.hpp — shared pieces of the batch and single-file command-line front-ends:
// argument helpers with the reference's parsing rules, the analyze_file flag -> AnalysisConfig
// mapping (examples/analyze_file.rs:190-680, in the same order, so later settings override
// earlier ones the same way), JSON string escaping as serde_json writes it, and the library's
// result/confidence calls.
#pragma once

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/stratum_hip.h"

namespace sdsp_cli {

using Args = std::vector<std::string>;

inline bool has(const Args& a, const char* name) {
    for (const auto& s : a)
        if (s == name) return true;
    return false;
}

// arg_value: the element after the first occurrence of `name`
inline bool arg_value(const Args& a, const char* name, std::string* out) {
    for (size_t i = 0; i < a.size(); i++)
        if (a[i] == name) {
            if (i + 1 >= a.size()) return false;
            *out = a[i + 1];
            return true;
        }
    return false;
}

// str::parse::<f32>: optional sign, decimal digits / exponent, inf / infinity / nan (any case)
inline bool parse_f32_str(const std::string& s, float* out) {
    if (s.empty()) return false;
    for (char c : s)
        if (std::isspace((unsigned char)c)) return false;
    if (s.size() > 1 && (s[0] == '0' || ((s[0] == '+' || s[0] == '-') && s.size() > 2 && s[1] == '0')) &&
        (s.find('x') != std::string::npos || s.find('X') != std::string::npos))
        return false;  // strtof would take hex floats; Rust does not
    char* end = nullptr;
    errno = 0;
    const float v = std::strtof(s.c_str(), &end);
    if (end != s.c_str() + s.size()) return false;
    *out = v;
    return true;
}

// str::parse::<usize>: optional '+', ASCII digits, no overflow
inline bool parse_usize_str(const std::string& s, uint64_t* out) {
    size_t i = (!s.empty() && s[0] == '+') ? 1 : 0;
    if (i >= s.size()) return false;
    uint64_t v = 0;
    for (; i < s.size(); i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        const uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (UINT64_MAX - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = v;
    return true;
}

inline bool parse_f32(const Args& a, const char* name, float* out) {
    std::string v;
    return arg_value(a, name, &v) && parse_f32_str(v, out);
}
inline bool parse_usize(const Args& a, const char* name, uint64_t* out) {
    std::string v;
    return arg_value(a, name, &v) && parse_usize_str(v, out);
}

// serde_json string encoding
inline std::string json_str(const std::string& s) {
    std::string o = "\"";
    for (unsigned char c : s) {
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            case '\b': o += "\\b"; break;
            case '\f': o += "\\f"; break;
            default:
                if (c < 0x20) {
                    char b[8];
                    std::snprintf(b, sizeof b, "\\u%04x", c);
                    o += b;
                } else {
                    o += (char)c;
                }
        }
    }
    return o + "\"";
}

inline std::string key_name(const sdsp_result& r) {
    char b[8];
    sdsp_key_name(r.key_mode, r.key_tonic, b, sizeof b);
    return b;
}

inline const char* tri(int8_t v) { return v < 0 ? "null" : v ? "true" : "false"; }

// Owned storage for the Vec fields a flag can set.
struct ConfigStore {
    std::vector<uint64_t> ms_lengths;
    std::vector<float> ms_weights;
};

// examples/analyze_file.rs:248-680 applied to `c` (which starts as AnalysisConfig::default()).
inline void apply_flags(const Args& a, sdsp_config* c, ConfigStore* st) {
    float x;
    uint64_t n;
    std::string s;
    if (has(a, "--no-preprocess")) {
        c->enable_normalization = 0;
        c->enable_silence_trimming = 0;
    }
    if (has(a, "--no-normalize")) c->enable_normalization = 0;
    if (has(a, "--no-trim")) c->enable_silence_trimming = 0;
    if (has(a, "--no-onset-consensus")) c->enable_onset_consensus = 0;
    if (has(a, "--force-legacy-bpm")) c->force_legacy_bpm = 1;
    if (has(a, "--bpm-fusion")) c->enable_bpm_fusion = 1;
    if (has(a, "--bpm-candidates")) c->emit_tempogram_candidates = 1;
    if (parse_usize(a, "--bpm-candidates-top", &n)) {
        c->emit_tempogram_candidates = 1;
        c->tempogram_candidates_top_n = n;
    }
    if (has(a, "--no-key-harmonic-mask")) c->enable_key_harmonic_mask = 0;
    if (parse_f32(a, "--key-harmonic-mask-power", &x)) c->key_harmonic_mask_power = x;
    if (has(a, "--key-hpss")) c->enable_key_hpss_harmonic = 1;
    if (has(a, "--no-key-hpss")) c->enable_key_hpss_harmonic = 0;
    if (parse_usize(a, "--key-hpss-frame-step", &n)) {
        c->enable_key_hpss_harmonic = 1;
        c->key_hpss_frame_step = n > 1 ? n : 1;
    }
    if (parse_usize(a, "--key-hpss-time-margin", &n)) {
        c->enable_key_hpss_harmonic = 1;
        c->key_hpss_time_margin = n;
    }
    if (parse_usize(a, "--key-hpss-freq-margin", &n)) {
        c->enable_key_hpss_harmonic = 1;
        c->key_hpss_freq_margin = n;
    }
    if (parse_f32(a, "--key-hpss-mask-power", &x)) {
        c->enable_key_hpss_harmonic = 1;
        c->key_hpss_mask_power = x;
    }
    if (has(a, "--no-key-stft-override")) c->enable_key_stft_override = 0;
    if (has(a, "--key-stft-override")) c->enable_key_stft_override = 1;
    if (parse_usize(a, "--key-stft-frame-size", &n)) {
        c->enable_key_stft_override = 1;
        c->key_stft_frame_size = n > 256 ? n : 256;
    }
    if (parse_usize(a, "--key-stft-hop-size", &n)) {
        c->enable_key_stft_override = 1;
        c->key_stft_hop_size = n > 1 ? n : 1;
    }
    if (has(a, "--no-key-log-freq")) c->enable_key_log_frequency = 0;
    if (has(a, "--key-log-freq")) c->enable_key_log_frequency = 1;
    if (has(a, "--no-key-beat-sync")) c->enable_key_beat_synchronous = 0;
    if (has(a, "--key-beat-sync")) c->enable_key_beat_synchronous = 1;
    if (has(a, "--no-key-multi-scale")) c->enable_key_multi_scale = 0;
    if (has(a, "--key-multi-scale")) c->enable_key_multi_scale = 1;
    if (arg_value(a, "--key-multi-scale-lengths", &s)) {  // comma-separated, all must parse
        std::vector<uint64_t> v;
        bool ok = true;
        size_t p = 0;
        while (ok) {
            const size_t q = s.find(',', p);
            std::string t = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
            while (!t.empty() && std::isspace((unsigned char)t.front())) t.erase(t.begin());
            while (!t.empty() && std::isspace((unsigned char)t.back())) t.pop_back();
            uint64_t u;
            ok = parse_usize_str(t, &u);
            if (ok) v.push_back(u);
            if (q == std::string::npos) break;
            p = q + 1;
        }
        if (ok) {
            st->ms_lengths = v;
            c->key_multi_scale_lengths = st->ms_lengths.data();
            c->key_multi_scale_lengths_len = st->ms_lengths.size();
            c->enable_key_multi_scale = 1;
        }
    }
    if (parse_usize(a, "--key-multi-scale-hop", &n)) {
        c->key_multi_scale_hop = n > 1 ? n : 1;
        c->enable_key_multi_scale = 1;
    }
    if (parse_f32(a, "--key-multi-scale-min-clarity", &x)) {
        c->key_multi_scale_min_clarity = x < 0.0f ? 0.0f : x > 1.0f ? 1.0f : x;
        c->enable_key_multi_scale = 1;
    }
    if (arg_value(a, "--key-multi-scale-weights", &s)) {
        std::vector<float> v;
        bool ok = true;
        size_t p = 0;
        while (ok) {
            const size_t q = s.find(',', p);
            std::string t = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
            while (!t.empty() && std::isspace((unsigned char)t.front())) t.erase(t.begin());
            while (!t.empty() && std::isspace((unsigned char)t.back())) t.pop_back();
            float f;
            ok = parse_f32_str(t, &f);
            if (ok) v.push_back(f);
            if (q == std::string::npos) break;
            p = q + 1;
        }
        if (ok) {
            st->ms_weights = v;
            c->key_multi_scale_weights = st->ms_weights.data();
            c->key_multi_scale_weights_len = st->ms_weights.size();
            c->enable_key_multi_scale = 1;
        }
    }
    if (has(a, "--key-template-temperley")) c->key_template_set = SDSP_TEMPLATES_TEMPERLEY;
    if (has(a, "--key-template-kk")) c->key_template_set = SDSP_TEMPLATES_KRUMHANSL_KESSLER;
    if (has(a, "--no-key-ensemble")) c->enable_key_ensemble = 0;
    if (has(a, "--key-ensemble")) c->enable_key_ensemble = 1;
    if (parse_f32(a, "--key-ensemble-kk-weight", &x)) {
        c->key_ensemble_kk_weight = x > 0.0f ? x : 0.0f;
        c->enable_key_ensemble = 1;
    }
    if (parse_f32(a, "--key-ensemble-temperley-weight", &x)) {
        c->key_ensemble_temperley_weight = x > 0.0f ? x : 0.0f;
        c->enable_key_ensemble = 1;
    }
    if (has(a, "--no-key-median")) c->enable_key_median = 0;
    if (has(a, "--key-median")) c->enable_key_median = 1;
    if (parse_usize(a, "--key-median-segment-length-frames", &n)) {
        c->key_median_segment_length_frames = n > 120 ? n : 120;
        c->enable_key_median = 1;
    }
    if (parse_usize(a, "--key-median-segment-hop-frames", &n)) {
        c->key_median_segment_hop_frames = n > 1 ? n : 1;
        c->enable_key_median = 1;
    }
    if (parse_usize(a, "--key-median-min-segments", &n)) {
        c->key_median_min_segments = n > 1 ? n : 1;
        c->enable_key_median = 1;
    }
    if (has(a, "--no-key-tuning")) c->enable_key_tuning_compensation = 0;
    if (parse_f32(a, "--key-tuning-max-semitones", &x)) c->key_tuning_max_abs_semitones = x;
    if (parse_usize(a, "--key-tuning-frame-step", &n)) c->key_tuning_frame_step = n;
    if (parse_f32(a, "--key-tuning-peak-rel-threshold", &x)) c->key_tuning_peak_rel_threshold = x;
    if (has(a, "--no-key-edge-trim")) c->enable_key_edge_trim = 0;
    if (parse_f32(a, "--key-edge-trim-fraction", &x)) c->key_edge_trim_fraction = x;
    if (has(a, "--no-key-segment-voting")) c->enable_key_segment_voting = 0;
    if (parse_usize(a, "--key-segment-len-frames", &n)) c->key_segment_len_frames = n;
    if (parse_usize(a, "--key-segment-hop-frames", &n)) c->key_segment_hop_frames = n;
    if (parse_f32(a, "--key-segment-min-clarity", &x)) c->key_segment_min_clarity = x;
    if (has(a, "--no-key-mode-heuristic")) c->enable_key_mode_heuristic = 0;
    if (has(a, "--key-mode-heuristic")) c->enable_key_mode_heuristic = 1;
    if (parse_f32(a, "--key-mode-third-margin", &x)) {
        c->enable_key_mode_heuristic = 1;
        c->key_mode_third_ratio_margin = x;
    }
    if (parse_f32(a, "--key-mode-flip-min-score-ratio", &x)) {
        c->enable_key_mode_heuristic = 1;
        c->key_mode_flip_min_score_ratio = x;
    }
    if (has(a, "--key-hpcp")) c->enable_key_hpcp = 1;
    if (parse_usize(a, "--key-hpcp-peaks", &n)) {
        c->enable_key_hpcp = 1;
        c->key_hpcp_peaks_per_frame = n;
    }
    if (parse_usize(a, "--key-hpcp-harmonics", &n)) {
        c->enable_key_hpcp = 1;
        c->key_hpcp_num_harmonics = n;
    }
    if (parse_f32(a, "--key-hpcp-harmonic-decay", &x)) {
        c->enable_key_hpcp = 1;
        c->key_hpcp_harmonic_decay = x;
    }
    if (parse_f32(a, "--key-hpcp-mag-power", &x)) {
        c->enable_key_hpcp = 1;
        c->key_hpcp_mag_power = x;
    }
    if (has(a, "--key-hpcp-whitening")) {
        c->enable_key_hpcp = 1;
        c->enable_key_hpcp_whitening = 1;
    }
    if (parse_usize(a, "--key-hpcp-whitening-smooth-bins", &n)) {
        c->enable_key_hpcp = 1;
        c->enable_key_hpcp_whitening = 1;
        c->key_hpcp_whitening_smooth_bins = n > 3 ? n : 3;
    }
    if (has(a, "--no-key-minor-harmonic-bonus")) c->enable_key_minor_harmonic_bonus = 0;
    if (has(a, "--key-minor-harmonic-bonus")) c->enable_key_minor_harmonic_bonus = 1;
    if (parse_f32(a, "--key-minor-leading-tone-bonus-weight", &x)) {
        c->enable_key_minor_harmonic_bonus = 1;
        c->key_minor_leading_tone_bonus_weight = x;
    }
    if (has(a, "--no-key-hpcp-bass")) c->enable_key_hpcp_bass_blend = 0;
    if (parse_f32(a, "--key-hpcp-bass-fmin-hz", &x)) {
        c->enable_key_hpcp_bass_blend = 1;
        c->key_hpcp_bass_fmin_hz = x;
    }
    if (parse_f32(a, "--key-hpcp-bass-fmax-hz", &x)) {
        c->enable_key_hpcp_bass_blend = 1;
        c->key_hpcp_bass_fmax_hz = x;
    }
    if (parse_f32(a, "--key-hpcp-bass-weight", &x)) {
        c->enable_key_hpcp_bass_blend = 1;
        c->key_hpcp_bass_weight = x;
    }
    if (has(a, "--no-key-spec-smooth")) c->enable_key_spectrogram_time_smoothing = 0;
    if (parse_usize(a, "--key-spec-smooth-margin", &n)) c->key_spectrogram_smooth_margin = n;
    if (has(a, "--no-key-frame-weighting")) c->enable_key_frame_weighting = 0;
    if (parse_f32(a, "--key-min-tonalness", &x)) c->key_min_tonalness = x;
    if (parse_f32(a, "--key-tonalness-power", &x)) c->key_tonalness_power = x;
    if (parse_f32(a, "--key-energy-power", &x)) c->key_energy_power = x;
    if (has(a, "--no-tempogram-multi-res")) c->enable_tempogram_multi_resolution = 0;
    struct MrF {
        const char* flag;
        float* field;
    } mrf[] = {{"--multi-res-w512", &c->tempogram_multi_res_w512},
               {"--multi-res-w256", &c->tempogram_multi_res_w256},
               {"--multi-res-w1024", &c->tempogram_multi_res_w1024},
               {"--multi-res-structural-discount", &c->tempogram_multi_res_structural_discount},
               {"--multi-res-double-time-512-factor", &c->tempogram_multi_res_double_time_512_factor},
               {"--multi-res-margin-threshold", &c->tempogram_multi_res_margin_threshold}};
    if (parse_usize(a, "--multi-res-top-k", &n)) {
        c->enable_tempogram_multi_resolution = 1;
        c->tempogram_multi_res_top_k = n;
    }
    for (auto& m : mrf)
        if (parse_f32(a, m.flag, &x)) {
            c->enable_tempogram_multi_resolution = 1;
            *m.field = x;
        }
    if (has(a, "--multi-res-human-prior")) {
        c->enable_tempogram_multi_resolution = 1;
        c->tempogram_multi_res_use_human_prior = 1;
    }
    if (has(a, "--no-tempogram-percussive")) c->enable_tempogram_percussive_fallback = 0;
    if (has(a, "--no-tempogram-band-fusion")) c->enable_tempogram_band_fusion = 0;
    if (has(a, "--band-score-fusion")) c->tempogram_band_seed_only = 0;
    if (has(a, "--no-tempogram-mel-novelty")) c->enable_tempogram_mel_novelty = 0;
    uint64_t tid;
    if (arg_value(a, "--debug-track-id", &s) && parse_usize_str(s, &tid) && tid <= UINT32_MAX) {
        c->has_debug_track_id = 1;
        c->debug_track_id = (uint32_t)tid;
        c->has_debug_gt_bpm = parse_f32(a, "--debug-gt-bpm", &x) ? 1 : 0;
        if (c->has_debug_gt_bpm) c->debug_gt_bpm = x;
    }
    struct F {
        const char* flag;
        float* field;
    } ff[] = {{"--band-low-max-hz", &c->tempogram_band_low_max_hz},
              {"--band-mid-max-hz", &c->tempogram_band_mid_max_hz},
              {"--band-high-max-hz", &c->tempogram_band_high_max_hz},
              {"--band-w-full", &c->tempogram_band_w_full},
              {"--band-w-low", &c->tempogram_band_w_low},
              {"--band-w-mid", &c->tempogram_band_w_mid},
              {"--band-w-high", &c->tempogram_band_w_high}};
    for (auto& f : ff)
        if (parse_f32(a, f.flag, &x)) *f.field = x;
    if (parse_usize(a, "--superflux-max-filter-bins", &n)) c->tempogram_superflux_max_filter_bins = n;
    if (parse_f32(a, "--band-support-threshold", &x)) c->tempogram_band_support_threshold = x;
    if (parse_f32(a, "--band-consensus-bonus", &x)) c->tempogram_band_consensus_bonus = x;
    if (parse_usize(a, "--mel-n-mels", &n)) c->tempogram_mel_n_mels = n;
    if (parse_f32(a, "--mel-fmin-hz", &x)) c->tempogram_mel_fmin_hz = x;
    if (parse_f32(a, "--mel-fmax-hz", &x)) c->tempogram_mel_fmax_hz = x;
    if (parse_usize(a, "--mel-max-filter-bins", &n)) c->tempogram_mel_max_filter_bins = n;
    if (parse_f32(a, "--mel-weight", &x)) c->tempogram_mel_weight = x;
    if (parse_f32(a, "--novelty-w-spectral", &x)) c->tempogram_novelty_w_spectral = x;
    if (parse_f32(a, "--novelty-w-energy", &x)) c->tempogram_novelty_w_energy = x;
    if (parse_f32(a, "--novelty-w-hfc", &x)) c->tempogram_novelty_w_hfc = x;
    if (parse_usize(a, "--novelty-local-mean-window", &n)) c->tempogram_novelty_local_mean_window = n;
    if (parse_usize(a, "--novelty-smooth-window", &n)) c->tempogram_novelty_smooth_window = n;
    F lf[] = {{"--legacy-preferred-min", &c->legacy_bpm_preferred_min},
              {"--legacy-preferred-max", &c->legacy_bpm_preferred_max},
              {"--legacy-soft-min", &c->legacy_bpm_soft_min},
              {"--legacy-soft-max", &c->legacy_bpm_soft_max},
              {"--legacy-mul-preferred", &c->legacy_bpm_conf_mul_preferred},
              {"--legacy-mul-soft", &c->legacy_bpm_conf_mul_soft},
              {"--legacy-mul-extreme", &c->legacy_bpm_conf_mul_extreme}};
    for (auto& f : lf)
        if (parse_f32(a, f.flag, &x)) *f.field = x;
}

}  // namespace sdsp_cli
