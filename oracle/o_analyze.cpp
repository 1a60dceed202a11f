// o_analyze.cpp — analyze_audio orchestration + the oracle's C API (TEST INFRASTRUCTURE).
//
// Follows src/lib.rs:86-1635 with AnalysisConfig::default() (src/config.rs:594-744) and the opt-in
// branches (normalisation methods, HPSS onsets and the percussive fallback, the legacy-BPM output
// paths, key scoring options, chroma front-ends).  Only degenerate sizes raise NotImplemented.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <sstream>

#include "oracle_internal.hpp"

using namespace orc;

extern "C" void sdsp_oracle_config_default(sdsp_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->min_amplitude_db = -40.0f;
    c->normalization = SDSP_NORM_PEAK;
    c->enable_normalization = 1;
    c->enable_silence_trimming = 1;
    c->enable_onset_consensus = 1;
    c->onset_threshold_percentile = 0.80f;
    c->onset_consensus_tolerance_ms = 50;
    for (int i = 0; i < 4; i++) c->onset_consensus_weights[i] = 0.25f;
    c->enable_hpss_onsets = 0;
    c->hpss_margin = 10;
    c->force_legacy_bpm = 0;
    c->enable_bpm_fusion = 0;
    c->enable_legacy_bpm_guardrails = 1;
    c->enable_tempogram_multi_resolution = 1;
    c->tempogram_multi_res_top_k = 25;
    c->tempogram_multi_res_w512 = 0.45f;
    c->tempogram_multi_res_w256 = 0.35f;
    c->tempogram_multi_res_w1024 = 0.20f;
    c->tempogram_multi_res_structural_discount = 0.85f;
    c->tempogram_multi_res_double_time_512_factor = 0.92f;
    c->tempogram_multi_res_margin_threshold = 0.08f;
    c->tempogram_multi_res_use_human_prior = 0;
    c->enable_tempogram_percussive_fallback = 0;
    c->enable_tempogram_band_fusion = 1;
    c->tempogram_band_low_max_hz = 200.0f;
    c->tempogram_band_mid_max_hz = 2000.0f;
    c->tempogram_band_high_max_hz = 8000.0f;
    c->tempogram_band_w_full = 0.40f;
    c->tempogram_band_w_low = 0.25f;
    c->tempogram_band_w_mid = 0.20f;
    c->tempogram_band_w_high = 0.15f;
    c->tempogram_band_seed_only = 1;
    c->tempogram_band_support_threshold = 0.25f;
    c->tempogram_band_consensus_bonus = 0.08f;
    c->tempogram_novelty_w_spectral = 0.30f;
    c->tempogram_novelty_w_energy = 0.35f;
    c->tempogram_novelty_w_hfc = 0.35f;
    c->tempogram_novelty_local_mean_window = 16;
    c->tempogram_novelty_smooth_window = 5;
    c->debug_top_n = 5;
    c->enable_tempogram_mel_novelty = 1;
    c->tempogram_mel_n_mels = 40;
    c->tempogram_mel_fmin_hz = 30.0f;
    c->tempogram_mel_fmax_hz = 8000.0f;
    c->tempogram_mel_max_filter_bins = 2;
    c->tempogram_mel_weight = 0.15f;
    c->tempogram_superflux_max_filter_bins = 4;
    c->emit_tempogram_candidates = 0;
    c->tempogram_candidates_top_n = 10;
    c->legacy_bpm_preferred_min = 72.0f;
    c->legacy_bpm_preferred_max = 168.0f;
    c->legacy_bpm_soft_min = 60.0f;
    c->legacy_bpm_soft_max = 210.0f;
    c->legacy_bpm_conf_mul_preferred = 1.30f;
    c->legacy_bpm_conf_mul_soft = 0.70f;
    c->legacy_bpm_conf_mul_extreme = 0.01f;
    c->min_bpm = 40.0f;
    c->max_bpm = 240.0f;
    c->bpm_resolution = 1.0f;
    c->frame_size = 2048;
    c->hop_size = 512;
    c->center_frequency = 440.0f;
    c->soft_chroma_mapping = 1;
    c->soft_mapping_sigma = 0.5f;
    c->chroma_sharpening_power = 1.0f;
    c->enable_key_spectrogram_time_smoothing = 1;
    c->key_spectrogram_smooth_margin = 12;
    c->enable_key_frame_weighting = 1;
    c->key_min_tonalness = 0.0f;
    c->key_tonalness_power = 2.0f;
    c->key_energy_power = 0.50f;
    c->enable_key_harmonic_mask = 1;
    c->key_harmonic_mask_power = 2.0f;
    c->enable_key_hpss_harmonic = 0;
    c->key_hpss_frame_step = 4;
    c->key_hpss_time_margin = 8;
    c->key_hpss_freq_margin = 8;
    c->key_hpss_mask_power = 2.0f;
    c->enable_key_stft_override = 1;
    c->key_stft_frame_size = 8192;
    c->key_stft_hop_size = 512;
    c->key_template_set = SDSP_TEMPLATES_KRUMHANSL_KESSLER;
    c->key_ensemble_kk_weight = 0.5f;
    c->key_ensemble_temperley_weight = 0.5f;
    c->key_median_segment_length_frames = 480;
    c->key_median_segment_hop_frames = 120;
    c->key_median_min_segments = 3;
    static const uint64_t ms_len[3] = {120, 360, 720};
    c->key_multi_scale_lengths = ms_len;
    c->key_multi_scale_lengths_len = 3;
    c->key_multi_scale_hop = 60;
    c->key_multi_scale_min_clarity = 0.20f;
    c->key_multi_scale_weights = nullptr;
    c->key_multi_scale_weights_len = 0;
    c->key_tuning_max_abs_semitones = 0.08f;
    c->key_tuning_frame_step = 20;
    c->key_tuning_peak_rel_threshold = 0.35f;
    c->key_edge_trim_fraction = 0.15f;
    c->enable_key_segment_voting = 1;
    c->key_segment_len_frames = 1024;
    c->key_segment_hop_frames = 512;
    c->key_segment_min_clarity = 0.20f;
    c->key_mode_third_ratio_margin = 0.00f;
    c->key_mode_flip_min_score_ratio = 0.60f;
    c->enable_key_hpcp = 1;
    c->key_hpcp_peaks_per_frame = 24;
    c->key_hpcp_num_harmonics = 4;
    c->key_hpcp_harmonic_decay = 0.60f;
    c->key_hpcp_mag_power = 0.50f;
    c->enable_key_hpcp_whitening = 0;
    c->key_hpcp_whitening_smooth_bins = 31;
    c->enable_key_hpcp_bass_blend = 0;
    c->key_hpcp_bass_fmin_hz = 55.0f;
    c->key_hpcp_bass_fmax_hz = 300.0f;
    c->key_hpcp_bass_weight = 0.35f;
    c->enable_key_minor_harmonic_bonus = 0;
    c->key_minor_leading_tone_bonus_weight = 0.2f;
}

namespace {

struct Out {
    float bpm = 0, bpm_conf = 0;
    int key_mode = 0;
    uint32_t key_tonic = 0;
    float key_conf = 0, key_clarity = 0, stability = 0, duration = 0, onset_consensus = 0;
    std::vector<float> beats, downbeats;
    std::vector<std::string> warnings;
    uint32_t flags = 0;
    int8_t mr_trig = -1, mr_used = -1, perc_trig = -1, perc_used = -1;
    bool has_cands = false;
    std::vector<TempoCand> cands;
};

[[noreturn]] void not_impl(const char* what) { fail(SDSP_ERR_NOT_IMPLEMENTED, std::string("oracle: ") + what); }

std::string fmt2(float v) {
    char b[64];
    std::snprintf(b, sizeof b, "%.2f", (double)v);
    return b;
}

void analyze(const float* samples, size_t n, uint32_t sr, const sdsp_config& c, Out& o, Trace& tr) {
    if (n == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty audio samples");  // lib.rs:100-110
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Invalid sample rate");
    std::vector<float> x(samples, samples + n);
    if (c.enable_normalization) {  // lib.rs:116-127
        if (c.normalization == SDSP_NORM_RMS)
            normalize_rms(x, -14.0f, 1.0f);
        else if (c.normalization == SDSP_NORM_LOUDNESS)
            normalize_lufs(x, sr, -14.0f, 1.0f);
        else
            normalize_peak(x, 1.0f);
    }
    size_t ts = 0, te = x.size();
    if (c.enable_silence_trimming) detect_and_trim(x, sr, c.min_amplitude_db, 500, c.frame_size, &ts, &te);
    tr.trim_start = ts;
    tr.trim_end = te;
    std::vector<float> trim(x.begin() + (long)ts, x.begin() + (long)te);
    if (trim.empty()) fail(SDSP_ERR_PROCESSING, "Audio is entirely silent after trimming");
    const size_t FS = c.frame_size, HOP = c.hop_size;
    if (FS == 0 || (FS & (FS - 1))) not_impl("non power-of-two frame_size");

    std::vector<size_t> energy = energy_flux_onsets(trim.data(), trim.size(), FS, HOP, -20.0f);  // :154-159
    tr.energy_onsets = energy;
    Spec mags = compute_stft(trim.data(), trim.size(), FS, HOP);  // :166
    std::vector<size_t> on_legacy = energy, on_beat = energy;
    // HPSS percussive component of the base spectrogram (hpss.rs:71-172): shared by the HPSS onsets
    // (:222-236) and the percussive tempogram fallback (:587-683), which decompose the same input
    Spec hp_H, hp_P;
    int hp_state = 0;  // 0 not computed, 1 ok, -1 failed
    auto percussive = [&]() -> const Spec* {
        if (hp_state == 0) {
            try {
                hpss_decompose(mags, (size_t)c.hpss_margin, &hp_H, &hp_P);
                hp_state = 1;
            } catch (const AErr&) {
                hp_state = -1;
            }
        }
        return hp_state == 1 ? &hp_P : nullptr;
    };
    if (c.enable_onset_consensus && !mags.empty()) {  // :176-291
        auto to_samples = [&](const std::vector<size_t>& fr) {
            std::vector<size_t> s;
            for (size_t f : fr) {
                const size_t v = f * HOP;
                if (v < trim.size()) s.push_back(v);
            }
            std::sort(s.begin(), s.end());
            s.erase(std::unique(s.begin(), s.end()), s.end());
            return s;
        };
        std::vector<size_t> lists[4];
        lists[0] = energy;
        try {
            lists[1] = to_samples(spectral_flux_onsets(mags, c.onset_threshold_percentile));
        } catch (const AErr&) {
        }
        try {
            lists[2] = to_samples(hfc_onsets(mags, sr, c.onset_threshold_percentile));
        } catch (const AErr&) {
        }
        if (c.enable_hpss_onsets) {
            try {
                if (const Spec* p = percussive()) lists[3] = to_samples(hpss_onsets(*p, c.onset_threshold_percentile));
            } catch (const AErr&) {
            }
        }
        tr.spectral_onsets = lists[1];
        tr.hfc_onsets = lists[2];
        try {
            auto cands = vote_onsets(lists, c.onset_consensus_weights, c.onset_consensus_tolerance_ms, sr);
            std::vector<size_t> strong, any;
            for (auto& cd : cands) {
                if (cd.voted_by >= 2) strong.push_back(cd.time_samples);
                any.push_back(cd.time_samples);
            }
            std::sort(strong.begin(), strong.end());
            strong.erase(std::unique(strong.begin(), strong.end()), strong.end());
            std::sort(any.begin(), any.end());
            any.erase(std::unique(any.begin(), any.end()), any.end());
            std::vector<size_t>& chosen = !strong.empty() ? strong : any;
            if (!chosen.empty()) {
                on_legacy = chosen;
                on_beat = chosen;
            }
        } catch (const AErr&) {
        }
    }
    tr.chosen_onsets = on_beat;

    // legacy (:294-329) — errors propagate
    BpmEstimate legacy{};
    bool has_legacy = false;
    if (on_legacy.size() >= 2) {
        Guardrails g{c.legacy_bpm_preferred_min, c.legacy_bpm_preferred_max, c.legacy_bpm_soft_min,
                     c.legacy_bpm_soft_max, c.legacy_bpm_conf_mul_preferred, c.legacy_bpm_conf_mul_soft,
                     c.legacy_bpm_conf_mul_extreme};
        has_legacy = estimate_bpm_legacy(on_legacy, sr, HOP, c.min_bpm, c.max_bpm, c.bpm_resolution,
                                         c.enable_legacy_bpm_guardrails ? &g : nullptr, &legacy);
    }
    tr.has_legacy = has_legacy;
    tr.legacy = legacy;

    // tempogram (:337-812)
    BandCfg band{(bool)c.enable_tempogram_band_fusion,
                 c.tempogram_band_low_max_hz,
                 c.tempogram_band_mid_max_hz,
                 c.tempogram_band_high_max_hz,
                 c.tempogram_band_w_full,
                 c.tempogram_band_w_low,
                 c.tempogram_band_w_mid,
                 c.tempogram_band_w_high,
                 (bool)c.tempogram_band_seed_only,
                 c.tempogram_band_support_threshold,
                 c.tempogram_band_consensus_bonus,
                 (bool)c.enable_tempogram_mel_novelty,
                 (size_t)c.tempogram_mel_n_mels,
                 c.tempogram_mel_fmin_hz,
                 c.tempogram_mel_fmax_hz,
                 (size_t)c.tempogram_mel_max_filter_bins,
                 c.tempogram_mel_weight,
                 c.tempogram_novelty_w_spectral,
                 c.tempogram_novelty_w_energy,
                 c.tempogram_novelty_w_hfc,
                 (size_t)c.tempogram_novelty_local_mean_window,
                 (size_t)c.tempogram_novelty_smooth_window,
                 (size_t)c.tempogram_superflux_max_filter_bins};
    const bool use_aux = c.enable_tempogram_band_fusion || c.enable_tempogram_mel_novelty ||
                         c.tempogram_band_consensus_bonus > 0.0f;
    bool has_tg = false;
    BpmEstimate tg{};
    if (!c.force_legacy_bpm && !mags.empty()) {
        const BandCfg* bp = use_aux ? &band : nullptr;
        auto run_impl = [&](size_t top_n, BpmEstimate* e, std::vector<TempoCand>* cands) -> bool {
            try {
                tempogram_impl(mags, sr, (uint32_t)HOP, c.min_bpm, c.max_bpm, c.bpm_resolution, bp, e, cands);
            } catch (const AErr&) {
                return false;
            }
            if (top_n == 0)
                cands->clear();
            else if (cands->size() > top_n)
                cands->resize(top_n);
            return true;
        };
        if (c.enable_tempogram_multi_resolution) {
            const size_t base_top_n =
                std::max<size_t>(std::max<size_t>(c.tempogram_candidates_top_n, c.tempogram_multi_res_top_k), 10);
            BpmEstimate base;
            std::vector<TempoCand> base_c;
            if (run_impl(base_top_n, &base, &base_c)) {
                tr.base = base;
                tr.base_cands = base_c;
                const bool trap_low = base.bpm >= 55.0f && base.bpm <= 80.0f;
                const bool trap_high = base.bpm >= 170.0f && base.bpm <= 200.0f;
                auto support = [&](float bpm, float tol) {
                    float b = 0.0f;
                    for (auto& cd : base_c)
                        if (sd_absf(cd.bpm - bpm) <= tol) b = sd_maxf(b, cd.score);
                    return b;
                };
                const float tol = sd_maxf(2.0f, c.bpm_resolution);
                const float s_base = support(base.bpm, tol), s_2x = support(base.bpm * 2.0f, tol),
                            s_half = support(base.bpm * 0.5f, tol);
                const bool family = (s_2x > 0.0f && s_2x >= s_base * 0.90f) || (s_half > 0.0f && s_half >= s_base * 0.90f);
                const bool fold_into_trap = base.bpm * 2.0f >= 170.0f && base.bpm * 2.0f <= 200.0f;
                const bool weak = base.method_agreement == 0 || base.confidence < 0.06f;
                const bool ambiguous = trap_low || trap_high || family || (weak && fold_into_trap);
                o.mr_trig = ambiguous;
                tr.ambiguous = ambiguous;
                BpmEstimate chosen = base;
                std::vector<TempoCand> chosen_c = base_c;
                bool used = false;
                if (ambiguous) {
                    BpmEstimate mr;
                    std::vector<TempoCand> mr_c;
                    bool ok = true;
                    try {
                        multi_resolution(trim, sr, FS, c.min_bpm, c.max_bpm, c.bpm_resolution,
                                         (size_t)c.tempogram_multi_res_top_k, c.tempogram_multi_res_w512,
                                         c.tempogram_multi_res_w256, c.tempogram_multi_res_w1024,
                                         c.tempogram_multi_res_structural_discount,
                                         c.tempogram_multi_res_double_time_512_factor,
                                         c.tempogram_multi_res_margin_threshold,
                                         (bool)c.tempogram_multi_res_use_human_prior, &band, &mr, &mr_c);
                    } catch (const AErr&) {
                        ok = false;
                    }
                    if (ok) {
                        tr.ran_mr = true;
                        tr.mr = mr;
                        const float rel = base.bpm > 1e-6f ? sd_maxf(mr.bpm / base.bpm, base.bpm / mr.bpm) : 1.0f;
                        const bool fam = sd_absf(rel - 2.0f) < 0.05f || sd_absf(rel - 1.5f) < 0.05f ||
                                         sd_absf(rel - (4.0f / 3.0f)) < 0.05f;
                        const bool forbid = base.bpm <= 180.0f && mr.bpm > 180.0f;
                        const bool better =
                            !forbid && (mr.confidence >= (base.confidence + 0.05f) ||
                                        (mr.method_agreement > base.method_agreement &&
                                         mr.confidence >= base.confidence * 0.90f) ||
                                        ((trap_low || trap_high) && fam && mr.confidence >= base.confidence * 0.88f &&
                                         ((mr.bpm >= 70.0f && mr.bpm <= 180.0f) || base.bpm > 180.0f)));
                        if (better) {
                            chosen = mr;
                            chosen_c = mr_c;
                            used = true;
                        }
                    }
                }
                o.mr_used = used;
                tr.used_mr = used;
                o.perc_trig = ambiguous && trap_low;
                if (c.enable_tempogram_percussive_fallback && ambiguous && trap_low) {  // :587-679
                    const Spec* p = percussive();
                    BpmEstimate pe;
                    std::vector<TempoCand> pc;
                    bool ok = p != nullptr;
                    if (ok) {
                        try {
                            tempogram_impl(*p, sr, (uint32_t)HOP, c.min_bpm, c.max_bpm, c.bpm_resolution, bp, &pe, &pc);
                            if (pc.size() > base_top_n) pc.resize(base_top_n);
                        } catch (const AErr&) {
                            ok = false;
                        }
                    }
                    bool p_used = false;
                    if (ok) {
                        const float rel =
                            chosen.bpm > 1e-6f ? sd_maxf(pe.bpm / chosen.bpm, chosen.bpm / pe.bpm) : 1.0f;
                        const bool fam = sd_absf(rel - 2.0f) < 0.05f || sd_absf(rel - 1.5f) < 0.05f ||
                                         sd_absf(rel - (4.0f / 3.0f)) < 0.05f || sd_absf(rel - (3.0f / 2.0f)) < 0.05f ||
                                         sd_absf(rel - (2.0f / 3.0f)) < 0.05f || sd_absf(rel - (3.0f / 4.0f)) < 0.05f;
                        const bool forbid = chosen.bpm <= 180.0f && pe.bpm > 180.0f;
                        const bool base_low_trap = trap_low || base.bpm < 95.0f;
                        const bool in_common = pe.bpm >= 70.0f && pe.bpm <= 180.0f;
                        p_used = !forbid && fam && in_common &&
                                 (pe.confidence >= chosen.confidence + 0.04f ||
                                  (base_low_trap && pe.confidence >= chosen.confidence * 0.85f) ||
                                  (pe.method_agreement > chosen.method_agreement &&
                                   pe.confidence >= chosen.confidence * 0.92f));
                        if (p_used) {
                            chosen = pe;
                            chosen_c = pc;
                        }
                    }
                    o.perc_used = p_used;
                } else if (c.enable_tempogram_percussive_fallback) {
                    o.perc_used = 0;
                }
                if (c.emit_tempogram_candidates) {
                    o.has_cands = true;
                    o.cands = chosen_c;
                }
                has_tg = true;
                tg = chosen;
            }
        } else if (c.emit_tempogram_candidates) {
            BpmEstimate e;
            std::vector<TempoCand> cd;
            if (run_impl((size_t)c.tempogram_candidates_top_n, &e, &cd)) {
                o.has_cands = true;
                o.cands = cd;
                has_tg = true;
                tg = e;
            }
        } else {
            BpmEstimate e;
            std::vector<TempoCand> cd;
            if (run_impl(0, &e, &cd)) {
                has_tg = true;
                tg = e;
            }
        }
    }
    tr.has_tempogram = has_tg;

    // BPM selection (:814-900)
    float bpm = 0.0f, bconf = 0.0f;
    if (c.force_legacy_bpm) {
        if (has_legacy) bpm = legacy.bpm, bconf = legacy.confidence;
    } else if (c.enable_bpm_fusion) {
        const float t_bpm = has_tg ? tg.bpm : 0.0f, t_conf = has_tg ? tg.confidence : 0.0f;
        const float l_bpm = has_legacy ? legacy.bpm : 0.0f;
        const float l_conf = sd_clampf(has_legacy ? legacy.confidence : 0.0f, 0.0f, 1.0f);
        if (t_bpm <= 0.0f) {
            if (has_legacy) bpm = legacy.bpm, bconf = legacy.confidence;
        } else {
            float conf = sd_clampf(t_conf, 0.0f, 1.0f);
            bool agree = false;
            if (l_bpm > 0.0f) {
                const float d[5] = {sd_absf(l_bpm - t_bpm), sd_absf(l_bpm - (t_bpm * 0.5f)), sd_absf(l_bpm - (t_bpm * 2.0f)),
                                    sd_absf(l_bpm - (t_bpm * (2.0f / 3.0f))), sd_absf(l_bpm - (t_bpm * (3.0f / 2.0f)))};
                for (float v : d) agree |= v <= 2.0f;
            }
            if (agree)
                conf = sd_clampf(conf + 0.12f * l_conf, 0.0f, 1.0f);
            else if (l_bpm > 0.0f)
                conf = sd_clampf(conf * 0.90f, 0.0f, 1.0f);
            bpm = t_bpm;
            bconf = conf;
        }
    } else if (has_tg) {
        bpm = tg.bpm, bconf = tg.confidence;
    } else if (has_legacy) {
        bpm = legacy.bpm, bconf = legacy.confidence;
    }
    o.bpm = bpm;
    o.bpm_conf = bconf;

    // beat grid (:913-958)
    if (bpm > 0.0f && on_beat.size() >= 2) {
        std::vector<float> os;
        for (size_t s : on_beat) os.push_back((float)s / (float)sr);
        std::vector<float> beats, down;
        float stab = 0.0f;
        if (generate_beat_grid(bpm, bconf, os, sr, &beats, &down, &stab, &tr.beat)) {
            o.beats = beats;
            o.downbeats = down;
            o.stability = stab;
        }
    }

    // key (:961-1559)
    if (trim.size() >= FS) {
        const size_t kfft = c.enable_key_stft_override ? std::max<size_t>(c.key_stft_frame_size, 256) : FS;
        const size_t khop = c.enable_key_stft_override ? std::max<size_t>(c.key_stft_hop_size, 1) : HOP;
        if (kfft & (kfft - 1)) not_impl("non power-of-two key_stft_frame_size");
        Spec ks = c.enable_key_stft_override ? compute_stft(trim.data(), trim.size(), kfft, khop) : mags;
        if (!ks.empty()) {  // :1011-1060
            if (c.enable_key_hpss_harmonic)
                key_hpss_mask_inplace(ks, sr, kfft, 100.0f, 5000.0f, (size_t)c.key_hpss_frame_step,
                                      (size_t)c.key_hpss_time_margin, (size_t)c.key_hpss_freq_margin,
                                      c.key_hpss_mask_power);
            else if (c.enable_key_harmonic_mask)
                harmonic_mask_inplace(ks, (size_t)c.key_spectrogram_smooth_margin, c.key_harmonic_mask_power);
            else if (c.enable_key_spectrogram_time_smoothing)
                smooth_time_inplace(ks, (size_t)c.key_spectrogram_smooth_margin);
        }
        // log-frequency spectrogram (:1062-1095)
        std::vector<float> chroma, energies;
        bool use_log = false;
        if (c.enable_key_log_frequency && !ks.empty()) {
            use_log = log_freq_chroma(ks, sr, kfft, &chroma, &energies);
            if (!use_log) not_impl("degenerate key log-frequency range");
        }
        // tuning offset (:1097-1119)
        float tuning = 0.0f;
        if (c.enable_key_tuning_compensation && !ks.empty() && !use_log) {
            const float lim = sd_absf(c.key_tuning_max_abs_semitones);
            tuning = sd_clampf(estimate_tuning(ks, sr, kfft, 80.0f, 2000.0f, (size_t)c.key_tuning_frame_step,
                                               c.key_tuning_peak_rel_threshold),
                               -lim, lim);
        }
        tr.tuning = tuning;
        // chroma front-end dispatch (:1121-1198)
        if (c.enable_key_beat_synchronous && !o.beats.empty() && !use_log) {
            beat_sync_chroma(ks, sr, kfft, khop, o.beats, c.soft_chroma_mapping != 0, c.soft_mapping_sigma, tuning,
                             &chroma, &energies);
        } else if (use_log) {
            // chroma / energies computed above
        } else if (c.enable_key_hpcp) {
            HpcpCfg hc;
            hc.sigma = c.soft_mapping_sigma;
            hc.tuning = tuning;
            hc.peaks = (size_t)c.key_hpcp_peaks_per_frame;
            hc.harmonics = (size_t)c.key_hpcp_num_harmonics;
            hc.decay = c.key_hpcp_harmonic_decay;
            hc.mag_power = c.key_hpcp_mag_power;
            hc.whitening = c.enable_key_hpcp_whitening != 0;
            hc.whitening_bins = (size_t)c.key_hpcp_whitening_smooth_bins;
            hc.bass_blend = c.enable_key_hpcp_bass_blend != 0;
            hc.bass_fmin = c.key_hpcp_bass_fmin_hz;
            hc.bass_fmax = c.key_hpcp_bass_fmax_hz;
            hc.bass_weight = c.key_hpcp_bass_weight;
            hpcp_frames_x(ks, sr, kfft, hc, &chroma, &energies);
        } else {
            const float t = (c.enable_key_tuning_compensation && sd_absf(tuning) > 1e-6f) ? tuning : 0.0f;
            chroma_frames(ks, sr, kfft, c.soft_chroma_mapping != 0, c.soft_mapping_sigma, t, &chroma, &energies);
        }
        const size_t F_all = energies.size();
        if (c.chroma_sharpening_power > 1.0f)  // :1200-1208
            for (size_t f = 0; f < F_all; f++) sharpen_chroma_inplace(chroma.data() + f * 12, c.chroma_sharpening_power);
        if (F_all > 5) smooth_chroma_inplace(chroma, F_all, 5);  // :1211-1213
        tr.chroma = chroma;
        tr.energies = energies;
        // optional edge trim (:1215-1232): the middle of the frames
        size_t t0 = 0, F = F_all;
        if (c.enable_key_edge_trim && energies.size() == F_all && F_all >= 200) {
            const float frac = sd_clampf(c.key_edge_trim_fraction, 0.0f, 0.49f);
            const size_t st = (size_t)sd_roundf((float)F_all * frac);
            const size_t en = (size_t)sd_roundf((float)F_all * (1.0f - frac));
            if (en > st + 50 && en <= F_all) {
                t0 = st;
                F = en - st;
            }
        }
        if (t0 > 0 || F != F_all) {
            chroma.erase(chroma.begin(), chroma.begin() + (long)(t0 * 12));
            chroma.resize(F * 12);
            energies.erase(energies.begin(), energies.begin() + (long)t0);
            energies.resize(F);
        }
        // frame weights (:1236-1287)
        std::vector<float> weights;
        bool use_w = false;
        if (c.enable_key_frame_weighting && F > 0 && energies.size() == F) {
            std::vector<float> sorted(energies);
            std::stable_sort(sorted.begin(), sorted.end(), [](float a, float b) { return a < b; });
            const float median = sd_maxf(sorted[sorted.size() / 2], 1e-12f);
            weights.resize(F);
            for (size_t f = 0; f < F; f++) {
                const float* ch = chroma.data() + f * 12;
                float sum = 0.0f;
                for (int i = 0; i < 12; i++) sum += ch[i];
                float tonal = 0.0f;
                if (!(sum <= 1e-12f)) {
                    float ent = 0.0f;
                    for (int i = 0; i < 12; i++) {
                        const float p = ch[i] / sum;
                        if (p > 1e-12f) ent -= p * sd_logf(p);
                    }
                    const float maxent = sd_logf(12.0f);
                    tonal = sd_clampf(1.0f - (ent / maxent), 0.0f, 1.0f);
                }
                if (tonal < c.key_min_tonalness) tonal = 0.0f;
                const float e_norm = sd_maxf(energies[f] / median, 0.0f);
                const float w_t = sd_powf(tonal, sd_maxf(c.key_tonalness_power, 0.0f));
                const float w_e = sd_powf(e_norm, sd_maxf(c.key_energy_power, 0.0f));
                weights[f] = sd_maxf(w_t * w_e, 0.0f);
            }
            use_w = true;
            float sw = 0.0f;
            size_t used = 0;
            for (float w : weights) {
                sw += w;
                used += w > 0.0f;
            }
            if (sw <= 1e-12f || used < 10) use_w = false;
        }
        tr.weights = weights;
        tr.weights_used = use_w;
        float maj[12][12], mnr[12][12];
        key_templates(maj, mnr, c.key_template_set == SDSP_TEMPLATES_TEMPERLEY ? 1 : 0);
        ModeHeuristic mh;
        mh.on = c.enable_key_mode_heuristic || c.enable_key_minor_harmonic_bonus;
        mh.third_margin = c.key_mode_third_ratio_margin;
        mh.flip_ratio = c.enable_key_mode_heuristic ? c.key_mode_flip_min_score_ratio : 0.0f;
        mh.bonus = c.enable_key_minor_harmonic_bonus;
        mh.bonus_w = c.key_minor_leading_tone_bonus_weight;
        std::vector<size_t> ms_len;
        for (uint64_t i = 0; i < c.key_multi_scale_lengths_len; i++) ms_len.push_back((size_t)c.key_multi_scale_lengths[i]);
        std::vector<float> ms_w(c.key_multi_scale_weights, c.key_multi_scale_weights + c.key_multi_scale_weights_len);
        const float* wp = use_w ? weights.data() : nullptr;
        auto detect_full = [&]() {
            return mh.on ? detect_key_weighted_mode_heuristic(chroma.data(), F, wp, maj, mnr, mh)
                         : detect_key_weighted(chroma.data(), F, wp, maj, mnr);
        };
        try {
            KeyResult kr;
            float clarity;
            const size_t seg_len_cfg = (size_t)c.key_segment_len_frames;
            const size_t ms_min = ms_len.empty() ? 1 : *std::min_element(ms_len.begin(), ms_len.end());
            if (c.enable_key_ensemble) {  // :1289-1299
                kr = detect_key_ensemble(chroma.data(), F, wp, c.key_ensemble_kk_weight, c.key_ensemble_temperley_weight);
                clarity = key_clarity(kr.scores, 24);
            } else if (c.enable_key_multi_scale && !ms_len.empty() && F >= ms_min) {  // :1304-1330
                int used = 0;
                if (!detect_key_multi_scale(chroma.data(), F, wp, maj, mnr, ms_len, (size_t)c.key_multi_scale_hop,
                                            sd_clampf(c.key_multi_scale_min_clarity, 0.0f, 1.0f),
                                            ms_w.empty() ? nullptr : &ms_w, mh, &kr, &used))
                    kr = detect_full();
                tr.used_segments = used;
                clarity = key_clarity(kr.scores, 24);
            } else if (c.enable_key_segment_voting && F >= std::max<size_t>(seg_len_cfg, 1) && seg_len_cfg >= 120 &&
                c.key_segment_hop_frames >= 1) {
                const size_t seg_len = std::min(seg_len_cfg, F);
                const size_t hop = std::max<size_t>(std::min<size_t>((size_t)c.key_segment_hop_frames, seg_len), 1);
                const float min_cl = sd_clampf(c.key_segment_min_clarity, 0.0f, 1.0f);
                float acc[24] = {0};
                int used = 0;
                for (size_t st = 0; st + seg_len <= F; st += hop) {
                    KeyResult sr_ = mh.on ? detect_key_weighted_mode_heuristic(chroma.data() + st * 12, seg_len,
                                                                               wp ? wp + st : nullptr, maj, mnr, mh)
                                          : detect_key_weighted(chroma.data() + st * 12, seg_len, wp ? wp + st : nullptr,
                                                                maj, mnr);
                    const float cl = key_clarity(sr_.scores, 24);
                    if (g_key_trace) g_key_trace->push_back(cl);
                    if (cl >= min_cl) {
                        used++;
                        for (int i = 0; i < 24; i++) acc[sr_.order[i]] += sr_.scores[i] * cl;
                    }
                }
                tr.used_segments = used;
                if (used == 0) {
                    kr = detect_full();
                    clarity = key_clarity(kr.scores, 24);
                } else {
                    int idx[24];
                    for (int i = 0; i < 24; i++) idx[i] = i;
                    std::stable_sort(idx, idx + 24, [&](int a, int b) { return acc[b] < acc[a]; });
                    float sorted[24];
                    for (int i = 0; i < 24; i++) sorted[i] = acc[idx[i]];
                    kr.mode = idx[0] < 12 ? 0 : 1;
                    kr.tonic = (uint32_t)(idx[0] % 12);
                    const float bs = sorted[0], ss = sorted[1];
                    kr.confidence = bs > 0.0f ? sd_clampf((bs - ss) / bs, 0.0f, 1.0f) : 0.0f;
                    clarity = key_clarity(sorted, 24);
                }
            } else {
                kr = detect_full();
                clarity = key_clarity(kr.scores, 24);
            }
            o.key_mode = kr.mode;
            o.key_tonic = kr.tonic;
            o.key_conf = kr.confidence;
            o.key_clarity = clarity;
        } catch (const AErr&) {
            o.key_mode = 0, o.key_tonic = 0, o.key_conf = 0.0f, o.key_clarity = 0.0f;
        }
    }

    // warnings / flags (:1564-1589)
    if (bpm == 0.0f) o.warnings.push_back("BPM detection failed: insufficient onsets or estimation error");
    if (o.stability < 0.5f)
        o.warnings.push_back("Low beat grid stability: " + fmt2(o.stability) + " (may indicate tempo variation)");
    if (o.key_conf < 0.3f)
        o.warnings.push_back("Low key detection confidence: " + fmt2(o.key_conf) +
                             " (may indicate ambiguous or atonal music)");
    if (o.key_clarity < 0.2f) {
        o.warnings.push_back("Low key clarity: " + fmt2(o.key_clarity) + " (track may be atonal or have weak tonality)");
        o.flags |= SDSP_FLAG_WEAK_TONALITY;
    }
    o.duration = (float)trim.size() / (float)sr;
    o.onset_consensus = energy.empty() ? 0.0f : 1.0f;
}

thread_local std::string g_trace_json;

template <class T>
void jarr(std::ostringstream& s, const char* k, const std::vector<T>& v) {
    s << "\"" << k << "\":[";
    for (size_t i = 0; i < v.size(); i++) s << (i ? "," : "") << v[i];
    s << "],";
}

void set_trace(const Trace& t) {
    std::ostringstream s;
    s.precision(9);
    s << "{";
    s << "\"trim_start\":" << t.trim_start << ",\"trim_end\":" << t.trim_end << ",";
    jarr(s, "energy_onsets", t.energy_onsets);
    jarr(s, "spectral_onsets", t.spectral_onsets);
    jarr(s, "hfc_onsets", t.hfc_onsets);
    jarr(s, "chosen_onsets", t.chosen_onsets);
    s << "\"has_legacy\":" << t.has_legacy << ",\"legacy\":[" << t.legacy.bpm << "," << t.legacy.confidence << ","
      << t.legacy.method_agreement << "],";
    s << "\"has_tempogram\":" << t.has_tempogram << ",\"base\":[" << t.base.bpm << "," << t.base.confidence << ","
      << t.base.method_agreement << "],";
    s << "\"ambiguous\":" << t.ambiguous << ",\"ran_mr\":" << t.ran_mr << ",\"used_mr\":" << t.used_mr;
    s << ",\"mr\":[" << t.mr.bpm << "," << t.mr.confidence << "," << t.mr.method_agreement << "],";
    s << "\"base_cands\":[";
    for (size_t i = 0; i < t.base_cands.size(); i++)
        s << (i ? "," : "") << "[" << t.base_cands[i].bpm << "," << t.base_cands[i].score << ","
          << t.base_cands[i].fft_norm << "," << t.base_cands[i].autocorr_norm << "]";
    s << "],";
    s << "\"weights_used\":" << t.weights_used << ",\"used_segments\":" << t.used_segments << ",";
    s << "\"beat_variable\":" << t.beat.variable << ",\"beat_refined\":" << t.beat.refined
      << ",\"beats_per_bar\":" << t.beat.beats_per_bar << ",";
    // key-stage checksums (sums in double over the frame-major arrays)
    double cs = 0, cq = 0, es = 0, ws = 0;
    for (float v : t.chroma) cs += v, cq += (double)v * v;
    for (float v : t.energies) es += v;
    for (float v : t.weights) ws += v;
    s.precision(17);
    // non-finite sums (non-finite input) as the tokens Python's json accepts
    auto num = [](double v) -> std::string {
        if (v != v) return "NaN";
        if (v == INFINITY) return "Infinity";
        if (v == -INFINITY) return "-Infinity";
        std::ostringstream o;
        o.precision(17);
        o << v;
        return o.str();
    };
    s << "\"chroma_sum\":" << num(cs) << ",\"chroma_sq\":" << num(cq) << ",\"energy_sum\":" << num(es)
      << ",\"weights_sum\":" << num(ws) << ",";
    s << "\"n_key_frames\":" << t.energies.size();
    s << "}";
    g_trace_json = s.str();
}

char* dup_str(const std::string& s) {
    char* p = (char*)std::malloc(s.size() + 1);
    std::memcpy(p, s.c_str(), s.size() + 1);
    return p;
}

float* dup_f(const std::vector<float>& v) {
    if (v.empty()) return nullptr;
    float* p = (float*)std::malloc(v.size() * sizeof(float));
    std::memcpy(p, v.data(), v.size() * sizeof(float));
    return p;
}

}  // namespace

extern "C" {

int32_t sdsp_oracle_analyze(const float* samples, uint64_t n, uint32_t sr, const sdsp_config* cfg, sdsp_result* r,
                            char* err, uint64_t errlen) {
    std::memset(r, 0, sizeof(*r));
    auto t0 = std::chrono::steady_clock::now();
    Out o;
    Trace tr;
    try {
        analyze(samples, (size_t)n, sr, *cfg, o, tr);
    } catch (const AErr& e) {
        static const char* pre[6] = {"", "Invalid input: ", "Decoding error: ", "Processing error: ",
                                     "Not implemented: ", "Numerical error: "};
        std::string m = std::string(pre[e.code]) + e.msg;
        if (err && errlen) {
            std::snprintf(err, (size_t)errlen, "%s", m.c_str());
        }
        r->status = e.code;
        std::snprintf(r->error_message, sizeof r->error_message, "%s", m.c_str());
        set_trace(tr);
        return e.code;
    }
    set_trace(tr);
    r->bpm = o.bpm;
    r->bpm_confidence = o.bpm_conf;
    r->key_mode = o.key_mode;
    r->key_tonic = o.key_tonic;
    r->key_confidence = o.key_conf;
    r->key_clarity = o.key_clarity;
    r->beats = dup_f(o.beats);
    r->n_beats = o.beats.size();
    r->downbeats = dup_f(o.downbeats);
    r->n_downbeats = o.downbeats.size();
    r->bars = dup_f(o.downbeats);
    r->n_bars = o.downbeats.size();
    r->grid_stability = o.stability;
    r->duration_seconds = o.duration;
    r->sample_rate = sr;
    r->processing_time_ms =
        (float)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::snprintf(r->algorithm_version, sizeof r->algorithm_version, "0.1.0-alpha");
    r->onset_method_consensus = o.onset_consensus;
    r->methods_used = 7;
    r->flags = o.flags;
    r->n_warnings = o.warnings.size();
    if (!o.warnings.empty()) {
        r->warnings = (char**)std::malloc(o.warnings.size() * sizeof(char*));
        for (size_t i = 0; i < o.warnings.size(); i++) r->warnings[i] = dup_str(o.warnings[i]);
    }
    r->has_tempogram_candidates = o.has_cands;
    if (o.has_cands && !o.cands.empty()) {
        r->n_tempogram_candidates = o.cands.size();
        r->tempogram_candidates = (sdsp_tempo_candidate*)std::malloc(o.cands.size() * sizeof(sdsp_tempo_candidate));
        for (size_t i = 0; i < o.cands.size(); i++)
            r->tempogram_candidates[i] = {o.cands[i].bpm, o.cands[i].score, o.cands[i].fft_norm,
                                          o.cands[i].autocorr_norm, (uint8_t)o.cands[i].selected};
    }
    r->tempogram_multi_res_triggered = o.mr_trig;
    r->tempogram_multi_res_used = o.mr_used;
    r->tempogram_percussive_triggered = o.perc_trig;
    r->tempogram_percussive_used = o.perc_used;
    r->status = SDSP_OK;
    return SDSP_OK;
}

void sdsp_oracle_result_free(sdsp_result* r) {
    std::free(r->beats);
    std::free(r->downbeats);
    std::free(r->bars);
    for (uint64_t i = 0; i < r->n_warnings; i++) std::free(r->warnings[i]);
    std::free(r->warnings);
    std::free(r->tempogram_candidates);
    r->beats = r->downbeats = r->bars = nullptr;
    r->warnings = nullptr;
    r->tempogram_candidates = nullptr;
}

const char* sdsp_oracle_last_trace_json(void) { return g_trace_json.c_str(); }

// ---- stage probes used by tests/ ----
int64_t sdsp_oracle_stft(const float* x, uint64_t n, uint64_t nfft, uint64_t hop, float* out) {
    Spec s = compute_stft(x, (size_t)n, (size_t)nfft, (size_t)hop);
    if (out && !s.d.empty()) std::memcpy(out, s.d.data(), s.d.size() * sizeof(float));
    return (int64_t)s.frames;
}

void sdsp_oracle_rfft(const float* x, uint64_t n, float* out_interleaved) {
    std::vector<Cx> X;
    rfft(x, (size_t)n, X);
    std::memcpy(out_interleaved, X.data(), X.size() * sizeof(Cx));
}

void sdsp_oracle_fft(float* io_interleaved, uint64_t M) {
    std::vector<Cx> x((size_t)M);
    std::memcpy(x.data(), io_interleaved, (size_t)M * sizeof(Cx));
    fft_complex(x);
    std::memcpy(io_interleaved, x.data(), (size_t)M * sizeof(Cx));
}

// combined full-band novelty of an STFT magnitude array (frames x bins), default band cfg
int64_t sdsp_oracle_novelty_full(const float* mags, uint64_t frames, uint64_t bins, uint32_t sr, float* out) {
    Spec s;
    s.frames = (size_t)frames;
    s.bins = (size_t)bins;
    s.d.assign(mags, mags + frames * bins);
    BandCfg b{true, 200, 2000, 8000, 0.4f, 0.25f, 0.2f, 0.15f, true, 0.25f, 0.08f, true, 40, 30.0f, 8000.0f, 2,
              0.15f, 0.30f, 0.35f, 0.35f, 16, 5, 4};
    auto v = combined_full_novelty(s, sr, b);
    if (out) std::memcpy(out, v.data(), v.size() * sizeof(float));
    return (int64_t)v.size();
}

// consensus.rs KATs: lists given as (n_i, ptr_i); writes (time, voted_by, conf) triples, returns count
int64_t sdsp_oracle_vote_onsets(const uint64_t* l0, uint64_t n0, const uint64_t* l1, uint64_t n1, const uint64_t* l2,
                                uint64_t n2, const uint64_t* l3, uint64_t n3, const float* w, uint32_t tol_ms,
                                uint32_t sr, uint64_t* times, uint32_t* voted, float* conf) {
    std::vector<size_t> L[4] = {std::vector<size_t>(l0, l0 + n0), std::vector<size_t>(l1, l1 + n1),
                                std::vector<size_t>(l2, l2 + n2), std::vector<size_t>(l3, l3 + n3)};
    try {
        auto c = vote_onsets(L, w, tol_ms, sr);
        for (size_t i = 0; i < c.size(); i++) {
            times[i] = c[i].time_samples;
            voted[i] = c[i].voted_by;
            conf[i] = c[i].confidence;
        }
        return (int64_t)c.size();
    } catch (const AErr& e) {
        return -(int64_t)e.code;
    }
}

// key_clarity.rs KAT probe
float sdsp_oracle_key_clarity(const float* scores, int32_t n) { return key_clarity(scores, n); }

// templates.rs probe: 24x12 (major 0..11 then minor 0..11)
void sdsp_oracle_key_templates(float* out) {
    float maj[12][12], mnr[12][12];
    key_templates(maj, mnr);
    std::memcpy(out, maj, sizeof maj);
    std::memcpy(out + 144, mnr, sizeof mnr);
}

// preprocessing::normalization::normalize with lib.rs's fixed config (target -14 LUFS, 1 dB
// headroom), in place; method 0 peak, 1 RMS, 2 LUFS.  Returns 0 or the error code (msg in err).
int32_t sdsp_oracle_normalize(int32_t method, float* x, uint64_t n, uint32_t sr, char* err, uint64_t errlen) {
    try {
        std::vector<float> v(x, x + n);
        if (method == 1)
            normalize_rms(v, -14.0f, 1.0f);
        else if (method == 2)
            normalize_lufs(v, sr, -14.0f, 1.0f);
        else
            normalize_peak(v, 1.0f);
        std::copy(v.begin(), v.end(), x);
        return 0;
    } catch (const AErr& e) {
        if (err && errlen) std::snprintf(err, errlen, "%s", e.msg.c_str());
        return e.code;
    }
}

// libm probes: op 0 ln, 1 exp, 2 cos, 3 log10, 4 log2, 5 pow(x, y), 6 sin, 7 atan2(x, y)
void sdsp_oracle_libm(int32_t op, const float* x, const float* y, float* out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        switch (op) {
            case 0: out[i] = sd_logf(x[i]); break;
            case 1: out[i] = sd_expf(x[i]); break;
            case 2: out[i] = sd_cosf(x[i]); break;
            case 3: out[i] = sd_log10f(x[i]); break;
            case 4: out[i] = sd_log2f(x[i]); break;
            case 6: out[i] = sd_sinf(x[i]); break;
            case 7: out[i] = sd_atan2f(x[i], y[i]); break;
            default: out[i] = sd_powf(x[i], y[i]); break;
        }
    }
}

}  // extern "C"
