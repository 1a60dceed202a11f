// o_key.cpp — key path (TEST INFRASTRUCTURE, see oracle_internal.hpp).
//
// Follows src/features/chroma/extractor.rs:529-680 (HPCP), :1097-1150 (driver + energies),
// :1246-1349 (time smoothing + harmonic mask); src/features/chroma/smoothing.rs:37-94;
// src/features/key/{detector.rs:68-313,984-1001; templates.rs:64-145; key_clarity.rs:51-93}.
#include <algorithm>

#include "oracle_internal.hpp"

namespace orc {
int g_block_energy = 0;
std::vector<float>* g_key_trace = nullptr;

// extractor.rs:1246-1290 + 1306-1349, streamed: the per-bin prefix sums are the reference's
// sequential f32 prefix (prefix[t+1] = prefix[t] + x), kept in a ring of 2*margin+2 rows.
void harmonic_mask_inplace(Spec& s, size_t margin, float power) {
    if (s.empty()) return;
    const size_t F = s.frames, B = s.bins;
    const float p = sd_maxf(power, 1.0f);
    const float eps = 1e-12f;
    if (margin == 0) {  // smooth_spectrogram_time returns the input unchanged -> h = x
        for (size_t t = 0; t < F; t++) {
            float* row = s.row(t);
            for (size_t b = 0; b < B; b++) {
                const float x = sd_maxf(row[b], 0.0f), h = sd_maxf(row[b], 0.0f);
                const float r = sd_maxf(x - h, 0.0f);
                const float hp = sd_powf(h, p), rp = sd_powf(r, p);
                row[b] = x * (hp / (hp + rp + eps));
            }
        }
        return;
    }
    const size_t R = 2 * margin + 2;
    std::vector<float> ring(R * B, 0.0f);  // ring[(i % R)*B + b] = prefix[i][b]
    for (size_t b = 0; b < B; b++) ring[b] = 0.0f;
    std::vector<float> hrow(B);
    for (size_t tin = 0; tin < F + margin; tin++) {
        if (tin < F) {
            const float* xr = s.row(tin);
            const float* pr = ring.data() + (tin % R) * B;
            float* nr = ring.data() + ((tin + 1) % R) * B;
            for (size_t b = 0; b < B; b++) nr[b] = pr[b] + xr[b];
        }
        if (tin < margin) continue;
        const size_t t = tin - margin;
        if (t >= F) break;
        const size_t st = t >= margin ? t - margin : 0;
        const size_t en = std::min(t + margin + 1, F);
        const float denom = (float)std::max<size_t>(en - st, 1);
        const float* pe = ring.data() + (en % R) * B;
        const float* ps = ring.data() + (st % R) * B;
        float* row = s.row(t);
        for (size_t b = 0; b < B; b++) {
            const float hm = (pe[b] - ps[b]) / denom;  // smooth_spectrogram_time output
            const float x = sd_maxf(row[b], 0.0f);
            const float h = sd_maxf(hm, 0.0f);
            const float r = sd_maxf(x - h, 0.0f);
            const float hp = sd_powf(h, p);
            const float rp = sd_powf(r, p);
            const float m = hp / (hp + rp + eps);
            row[b] = x * m;
        }
    }
}

// compiler-rt __powisf2 (Rust f32::powi with a runtime exponent)
static float powi_f(float a, int b) {
    const bool recip = b < 0;
    float r = 1.0f;
    while (true) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1.0f / r : r;
}

// extractor.rs:1097-1150 -> frame_to_hpcp_tuned_band (:529-680), whitening off, tuning 0,
// band [100, 5000] Hz.  Top-K peaks are taken in (magnitude desc, bin asc) order: the
// reference's select_nth_unstable_by leaves an implementation-defined order.
void hpcp_frames(const Spec& s, uint32_t sr, size_t fft_size, float sigma_in, size_t peaks_k, size_t harmonics,
                 float decay_in, float mag_power, std::vector<float>* chroma12, std::vector<float>* energies) {
    chroma12->assign(s.frames * 12, 0.0f);
    energies->assign(s.frames, 0.0f);
    if (s.empty()) return;
    const float fres = (float)sr / (float)fft_size;
    const float fmin = sd_maxf(100.0f, 20.0f);
    const float fmax = sd_minf(5000.0f, (float)sr / 2.0f);
    const float sigma = sd_maxf(sigma_in, 1e-6f);
    const size_t hmax = std::max<size_t>(harmonics, 1);
    const float decay = sd_clampf(decay_in, 0.0f, 1.0f);
    const float p = sd_clampf(mag_power, 0.05f, 1.0f);
    std::vector<std::pair<size_t, float>> peaks;
    for (size_t t = 0; t < s.frames; t++) {
        const float* m = s.row(t);
        float e = 0.0f;
        for (size_t b = 0; b < s.bins; b++) e += m[b] * m[b];
        (*energies)[t] = e;
        float* pc = chroma12->data() + t * 12;
        if (fmax <= fmin) continue;
        peaks.clear();
        for (size_t bin = 1; bin + 1 < s.bins; bin++) {
            const float freq = (float)bin * fres;
            if (freq < fmin) continue;
            if (freq > fmax) break;
            const float mv = m[bin], mp = m[bin - 1], mn = m[bin + 1];
            if (mv <= mp || mv < mn) continue;
            peaks.push_back({bin, mv});
        }
        if (peaks.empty()) continue;
        const size_t k = std::min(std::max<size_t>(peaks_k, 1), peaks.size());
        std::stable_sort(peaks.begin(), peaks.end(), [](auto& a, auto& b) { return b.second < a.second; });
        peaks.resize(k);
        for (auto& pk : peaks) {
            const float f0 = (float)pk.first * fres;
            if (f0 <= 0.0f) continue;
            const float w0 = sd_powf(sd_maxf(m[pk.first], 0.0f), p);
            if (w0 <= 0.0f) continue;
            for (size_t h = 1; h <= hmax; h++) {
                const float fh = f0 * (float)h;
                if (fh > fmax) break;
                if (fh < fmin) continue;
                const float semitone = 12.0f * sd_log2f(fh / 440.0f) + 57.0f - 0.0f;
                const float spc = sd_rem_euclid_f(semitone, 12.0f);
                const float ppc = sd_rem_euclid_f(sd_roundf(spc), 12.0f);
                const int32_t primary = sd_f2i32(ppc);
                const float hw = powi_f(decay, (int)h - 1) / (float)h;
                const float contrib = w0 * hw;
                for (int off = -1; off <= 1; off++) {
                    const int tc = (((primary + off) % 12) + 12) % 12;
                    float dist = sd_absf(spc - (float)tc);
                    dist = sd_minf(dist, 12.0f - dist);
                    const float wgt = sd_expf(-dist * dist / (2.0f * sigma * sigma));
                    pc[tc] += contrib * wgt;
                }
            }
        }
        float nsq = 0.0f;
        for (int i = 0; i < 12; i++) nsq += pc[i] * pc[i];
        const float norm = __builtin_sqrtf(nsq);
        if (norm > EPS)
            for (int i = 0; i < 12; i++) pc[i] /= norm;
    }
}

// smoothing.rs:37-94 (window forced odd; median = sorted[len/2])
void smooth_chroma_inplace(std::vector<float>& ch, size_t frames, size_t window) {
    if (frames == 0 || window <= 1) return;
    if (window % 2 == 0) window += 1;
    const int64_t half = (int64_t)window / 2;
    std::vector<float> out(ch.size());
    float vals[64];
    for (size_t t = 0; t < frames; t++) {
        for (int s = 0; s < 12; s++) {
            int n = 0;
            for (int64_t o = 0; o < (int64_t)window; o++) {
                const int64_t fi = (int64_t)t + (o - half);
                if (fi >= 0 && fi < (int64_t)frames) vals[n++] = ch[(size_t)fi * 12 + (size_t)s];
            }
            std::stable_sort(vals, vals + n, [](float a, float b) { return a < b; });
            out[t * 12 + (size_t)s] = vals[n / 2];
        }
    }
    ch.swap(out);
}

// templates.rs:64-145 (K-K) and :147-235 (Temperley): profiles rotated, then L2-normalised per
// key in rotated order
void key_templates(float maj[12][12], float min_[12][12], int template_set) {
    const float kM[12] = {6.35f, 2.23f, 3.48f, 2.33f, 4.38f, 4.09f, 2.52f, 5.19f, 2.39f, 3.66f, 2.29f, 2.88f};
    const float km[12] = {6.33f, 2.68f, 3.52f, 5.38f, 2.60f, 3.53f, 2.54f, 4.75f, 3.98f, 2.69f, 3.34f, 3.17f};
    const float tM[12] = {5.0f, 2.0f, 3.5f, 2.0f, 4.5f, 4.0f, 2.0f, 4.5f, 2.0f, 3.5f, 1.5f, 4.0f};
    const float tm[12] = {5.0f, 2.0f, 3.5f, 5.0f, 2.0f, 3.5f, 2.0f, 4.5f, 3.5f, 2.0f, 4.0f, 3.5f};
    const float* cM = template_set == 1 ? tM : kM;
    const float* cm = template_set == 1 ? tm : km;
    for (int k = 0; k < 12; k++)
        for (int s = 0; s < 12; s++) {
            maj[k][s] = cM[(s + 12 - k) % 12];
            min_[k][s] = cm[(s + 12 - k) % 12];
        }
    auto l2 = [](float* v) {
        float sq = 0.0f;
        for (int i = 0; i < 12; i++) sq += v[i] * v[i];
        const float n = __builtin_sqrtf(sq);
        if (n > 1e-12f)
            for (int i = 0; i < 12; i++) v[i] /= n;
    };
    for (int k = 0; k < 12; k++) {
        l2(maj[k]);
        l2(min_[k]);
    }
}

// detector.rs:984-1001
static float weighted_sum_dot(const float* ch, size_t frames, const float* w, const float* tpl) {
    float acc = 0.0f;
    for (size_t f = 0; f < frames; f++) {
        const float* c = ch + f * 12;
        if (w) {
            const float wt = w[f];
            if (wt > 0.0f) {
                float d = 0.0f;
                for (int i = 0; i < 12; i++) d += c[i] * tpl[i];
                acc += wt * d;
            }
        } else {
            float d = 0.0f;
            for (int i = 0; i < 12; i++) d += c[i] * tpl[i];
            acc += d;
        }
    }
    return acc;
}

// detector.rs:68-313.  The HashMap top-3 vote (:259-275) returns scores[0]'s key unless the
// top two scores tie exactly (then the reference itself is nondeterministic); we return scores[0].
KeyResult detect_key_weighted(const float* ch, size_t frames, const float* w, const float maj[12][12],
                              const float mnr[12][12]) {
    if (frames == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty chroma vectors");
    float sc[24];
    for (int k = 0; k < 12; k++) sc[k] = weighted_sum_dot(ch, frames, w, maj[k]);
    for (int k = 0; k < 12; k++) sc[12 + k] = weighted_sum_dot(ch, frames, w, mnr[k]);
    if (g_key_trace) g_key_trace->insert(g_key_trace->end(), sc, sc + 24);
    float mM = 0.0f, mm = 0.0f;
    for (int k = 0; k < 12; k++) mM = sd_maxf(mM, sc[k]);
    for (int k = 0; k < 12; k++) mm = sd_maxf(mm, sc[12 + k]);
    if (mM > 1e-9f && mm > 1e-9f) {
        for (int k = 0; k < 12; k++) sc[k] /= mM;
        for (int k = 0; k < 12; k++) sc[12 + k] /= mm;
    }
    // top key per mode: max_by -> LAST maximum
    int tM = 0, tm = 0;
    for (int k = 1; k < 12; k++)
        if (!(sc[k] < sc[tM])) tM = k;
    for (int k = 1; k < 12; k++)
        if (!(sc[12 + k] < sc[12 + tm])) tm = k;
    const float tMs = sc[tM], tms = sc[12 + tm];
    const int cof[12] = {0, 7, 2, 9, 4, 11, 6, 1, 8, 3, 10, 5};
    auto pos = [&](int tonic) {
        for (int i = 0; i < 12; i++)
            if (cof[i] == tonic) return i;
        return 12;
    };
    float rs[24];
    for (int i = 0; i < 24; i++) {
        rs[i] = sc[i];
        const bool major = i < 12;
        const int ref_t = major ? tM : tm;
        const float ref_s = major ? tMs : tms;
        if (ref_s > 1e-9f) {
            const int tp = pos(i % 12), rp = pos(ref_t);
            if (tp < 12 && rp < 12) {
                const int ad = tp > rp ? tp - rp : rp - tp;
                const int dist = std::min(ad, 12 - ad);
                if (dist <= 2) {
                    const float bonus = 0.20f * (1.0f - (float)dist * 0.5f);
                    rs[i] += ref_s * bonus;
                }
            }
        }
    }
    KeyResult r{};
    int idx[24];
    for (int i = 0; i < 24; i++) idx[i] = i;
    std::stable_sort(idx, idx + 24, [&](int a, int b) { return rs[b] < rs[a]; });
    for (int i = 0; i < 24; i++) {
        r.order[i] = idx[i];
        r.scores[i] = rs[idx[i]];
    }
    r.mode = idx[0] < 12 ? 0 : 1;
    r.tonic = (uint32_t)(idx[0] % 12);
    const float fs = r.scores[0];
    const float bo = r.scores[1];  // first entry whose key != final key
    r.confidence = fs > 0.0f ? sd_clampf((fs - bo) / fs, 0.0f, 1.0f) : 0.0f;
    return r;
}

// chroma/normalization.rs:41-65: x^p, L2-normalise (EPSILON 1e-10), else uniform 1/sqrt(12)
void sharpen_chroma_inplace(float* ch, float power) {
    float sq = 0.0f;
    for (int i = 0; i < 12; i++) {
        ch[i] = sd_powf(ch[i], power);
        sq += ch[i] * ch[i];
    }
    const float norm = __builtin_sqrtf(sq);
    if (norm > 1e-10f) {
        for (int i = 0; i < 12; i++) ch[i] /= norm;
    } else {
        const float u = 1.0f / __builtin_sqrtf(12.0f);
        for (int i = 0; i < 12; i++) ch[i] = u;
    }
}

// detector.rs:326-506.  `scores`/`order` of the result are the post-bonus table, stably re-sorted
// from the base result's order; mode/tonic/confidence are the (possibly mode-flipped) choice.
KeyResult detect_key_weighted_mode_heuristic(const float* ch, size_t frames, const float* w, const float maj[12][12],
                                             const float mnr[12][12], const ModeHeuristic& mh) {
    const KeyResult base = detect_key_weighted(ch, frames, w, maj, mnr);
    const float flip_ratio = sd_clampf(mh.flip_ratio, 0.0f, 1.0f);
    const bool mode_flip = flip_ratio > 0.0f;
    if (!mh.bonus && !mode_flip) return base;
    float avg[12] = {0};
    float wsum = 0.0f;
    if (!w) {
        for (size_t f = 0; f < frames; f++)
            for (int i = 0; i < 12; i++) avg[i] += ch[f * 12 + i];
        wsum = (float)frames;
    } else {
        for (size_t f = 0; f < frames; f++) {
            const float wt = w[f];
            if (wt <= 0.0f) continue;
            for (int i = 0; i < 12; i++) avg[i] += wt * ch[f * 12 + i];
            wsum += wt;
        }
    }
    if (wsum <= 1e-9f) return base;
    float sum = -0.0f;
    for (int i = 0; i < 12; i++) sum += avg[i];
    if (sum > 1e-9f)
        for (int i = 0; i < 12; i++) avg[i] /= sum;
    float sc[24];
    int ord[24];
    for (int i = 0; i < 24; i++) {
        sc[i] = base.scores[i];
        ord[i] = base.order[i];
    }
    if (mh.bonus) {
        const float bw = sd_maxf(mh.bonus_w, 0.0f);
        if (bw > 0.0f)
            for (int i = 0; i < 24; i++)
                if (ord[i] >= 12) {
                    const int tonic = ord[i] - 12;
                    const int lt = (tonic + 11) % 12, b7 = (tonic + 10) % 12;
                    sc[i] += wsum * bw * (avg[lt] - avg[b7]);
                }
    }
    {  // stable sort desc of the base-ordered table
        int idx[24];
        for (int i = 0; i < 24; i++) idx[i] = i;
        std::stable_sort(idx, idx + 24, [&](int a, int b) { return sc[b] < sc[a]; });
        float s2[24];
        int o2[24];
        for (int i = 0; i < 24; i++) {
            s2[i] = sc[idx[i]];
            o2[i] = ord[idx[i]];
        }
        for (int i = 0; i < 24; i++) {
            sc[i] = s2[i];
            ord[i] = o2[i];
        }
    }
    float major_s[12] = {0}, minor_s[12] = {0};
    for (int i = 0; i < 24; i++) (ord[i] < 12 ? major_s[ord[i]] : minor_s[ord[i] - 12]) = sc[i];
    const int best = ord[0];
    const int tonic = best % 12;
    const bool best_major = best < 12;
    const float p_min3 = avg[(tonic + 3) % 12], p_maj3 = avg[(tonic + 4) % 12];
    const float p_min6 = avg[(tonic + 8) % 12], p_maj6 = avg[(tonic + 9) % 12];
    const float p_min7 = avg[(tonic + 10) % 12], p_maj7 = avg[(tonic + 11) % 12];
    const float margin = sd_maxf(mh.third_margin, 0.0f);
    float minor_score = 0.0f, major_score = 0.0f;
    const float third = sd_absf(p_min3 - p_maj3);
    if (p_min3 > p_maj3 * (1.0f + margin))
        minor_score += third * 2.0f;
    else if (p_maj3 > p_min3 * (1.0f + margin))
        major_score += third * 2.0f;
    const float sixth = sd_absf(p_min6 - p_maj6);
    if (p_min6 > p_maj6 * (1.0f + margin))
        minor_score += sixth * 1.0f;
    else if (p_maj6 > p_min6 * (1.0f + margin))
        major_score += sixth * 1.0f;
    const float seventh = sd_absf(p_min7 - p_maj7);
    if (p_min7 > p_maj7 * (1.0f + margin))
        minor_score += seventh * 1.0f;
    else if (p_maj7 > p_min7 * (1.0f + margin))
        major_score += seventh * 1.0f;
    const float total = minor_score + major_score;
    const bool minor_pref = total > 1e-9f ? minor_score > major_score * (1.0f + margin * 0.5f) : false;
    const bool major_pref = total > 1e-9f ? major_score > minor_score * (1.0f + margin * 0.5f) : false;
    int chosen = best;
    if (mode_flip) {
        if (best_major && minor_pref) {
            const float sb = major_s[tonic], sa = minor_s[tonic];
            if (sb > 0.0f && sa >= sb * flip_ratio) chosen = 12 + tonic;
        } else if (!best_major && major_pref) {
            const float sb = minor_s[tonic], sa = major_s[tonic];
            if (sb > 0.0f && sa >= sb * flip_ratio) chosen = tonic;
        }
    }
    const float chosen_s = chosen < 12 ? major_s[chosen] : minor_s[chosen - 12];
    float best_other = 0.0f;
    for (int i = 0; i < 24; i++)
        if (ord[i] != chosen) best_other = sd_maxf(best_other, sc[i]);
    KeyResult r{};
    for (int i = 0; i < 24; i++) {
        r.scores[i] = sc[i];
        r.order[i] = ord[i];
    }
    r.mode = chosen < 12 ? 0 : 1;
    r.tonic = (uint32_t)(chosen % 12);
    r.confidence = chosen_s > 0.0f ? sd_clampf((chosen_s - best_other) / chosen_s, 0.0f, 1.0f) : 0.0f;
    return r;
}

static KeyResult from_table(const float acc[24]) {  // stable sort desc + (best - second) / best
    int idx[24];
    for (int i = 0; i < 24; i++) idx[i] = i;
    std::stable_sort(idx, idx + 24, [&](int a, int b) { return acc[b] < acc[a]; });
    KeyResult r{};
    for (int i = 0; i < 24; i++) {
        r.order[i] = idx[i];
        r.scores[i] = acc[idx[i]];
    }
    r.mode = idx[0] < 12 ? 0 : 1;
    r.tonic = (uint32_t)(idx[0] % 12);
    const float bs = r.scores[0], ss = r.scores[1];
    r.confidence = bs > 0.0f ? sd_clampf((bs - ss) / bs, 0.0f, 1.0f) : 0.0f;
    return r;
}

// detector.rs:881-978
KeyResult detect_key_ensemble(const float* ch, size_t frames, const float* w, float kk_weight, float temp_weight) {
    const float total = kk_weight + temp_weight;
    const float kk_norm = total > 1e-9f ? kk_weight / total : 0.5f;
    const float tp_norm = total > 1e-9f ? temp_weight / total : 0.5f;
    float km[12][12], kn[12][12], tm[12][12], tn[12][12];
    key_templates(km, kn, 0);
    key_templates(tm, tn, 1);
    const KeyResult a = detect_key_weighted(ch, frames, w, km, kn);
    const KeyResult b = detect_key_weighted(ch, frames, w, tm, tn);
    float sa[24], sb[24], comb[24];
    for (int i = 0; i < 24; i++) {
        sa[a.order[i]] = a.scores[i];
        sb[b.order[i]] = b.scores[i];
    }
    for (int k = 0; k < 24; k++) comb[k] = kk_norm * sa[k] + tp_norm * sb[k];
    return from_table(comb);
}

// detector.rs:546-719 (the fallback to full-track detection is the caller's)
bool detect_key_multi_scale(const float* ch, size_t frames, const float* w, const float maj[12][12],
                            const float mnr[12][12], const std::vector<size_t>& lengths, size_t hop_in, float min_cl,
                            const std::vector<float>* scale_w, const ModeHeuristic& mh, KeyResult* out,
                            int* used_segments) {
    float acc[24] = {0};
    float total_w = 0.0f;
    int used = 0;
    const size_t hop = std::max<size_t>(hop_in, 1);
    for (size_t si = 0; si < lengths.size(); si++) {
        const size_t len = lengths[si];
        if (len == 0 || len > frames) continue;
        const float sw = (scale_w && si < scale_w->size()) ? (*scale_w)[si] : 1.0f;
        if (sw <= 0.0f) continue;
        for (size_t st = 0; st + len <= frames; st += hop) {
            const KeyResult r = mh.on ? detect_key_weighted_mode_heuristic(ch + st * 12, len, w ? w + st : nullptr, maj,
                                                                           mnr, mh)
                                      : detect_key_weighted(ch + st * 12, len, w ? w + st : nullptr, maj, mnr);
            const float cl = key_clarity(r.scores, 24);
            if (cl >= min_cl) {
                used++;
                const float cw = cl * sw;
                total_w += cw;
                for (int i = 0; i < 24; i++) acc[r.order[i]] += r.scores[i] * cw;
            }
        }
    }
    *used_segments = used;
    if (used == 0 || total_w <= 1e-12f) return false;
    for (int k = 0; k < 24; k++) acc[k] /= total_w;
    *out = from_table(acc);
    return true;
}

// key_clarity.rs:51-93 (scores in the given order)
float key_clarity(const float* s, int n) {
    if (n < 2) return 0.0f;
    const float best = s[0];
    float sum = 0.0f;
    for (int i = 0; i < n; i++) sum += s[i];
    const float avg = sum / (float)n;
    float mn = s[0], mx = s[0];
    for (int i = 1; i < n; i++) {
        if (s[i] < mn) mn = s[i];  // min_by: first minimum
        if (!(s[i] < mx)) mx = s[i];
    }
    const float range = mx - mn;
    if (range > 1e-10f) return sd_clampf((best - avg) / range, 0.0f, 1.0f);
    return 0.0f;
}

}  // namespace orc

// ---- unit probes (tests only; tests/test_oracle_units_key.py) ----
using namespace orc;

extern "C" {

// detect_key_weighted (detector.rs:68-313) with K-K templates (KeyTemplates::new()); weights
// nullable (detect_key).  dims = the chroma vectors' length (the reference rejects != 12);
// n_weights = the weight slice length (rejected when != frames).  Outputs: key index
// (mode * 12 + tonic), confidence, the 24 refined scores in sorted order and their key indices
// (all_scores; top_keys = the first 3).
int32_t sdsp_oracle_detect_key(const float* chroma, uint64_t frames, uint64_t dims, const float* weights,
                               uint64_t n_weights, int32_t* key, float* conf, float* scores24, int32_t* keys24) {
    return (int32_t)probe_call([&]() -> int64_t {
        if (frames == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty chroma vectors");
        if (dims != 12) fail(SDSP_ERR_INVALID_INPUT, "Chroma vectors must have 12 elements");
        if (weights && n_weights != frames) fail(SDSP_ERR_INVALID_INPUT, "frame_weights length mismatch");
        float maj[12][12], mnr[12][12];
        key_templates(maj, mnr, 0);
        const KeyResult r = detect_key_weighted(chroma, frames, weights, maj, mnr);
        *key = r.mode * 12 + (int32_t)r.tonic;
        *conf = r.confidence;
        for (int i = 0; i < 24; i++) {
            scores24[i] = r.scores[i];
            keys24[i] = r.order[i];
        }
        return 0;
    });
}

// smooth_chroma (smoothing.rs:37-94, median) or smooth_chroma_average (:103-150): frames x 12
void sdsp_oracle_smooth_chroma(const float* ch, uint64_t frames, uint64_t window, int32_t average, float* out) {
    std::vector<float> v(ch, ch + frames * 12);
    if (!average) {
        smooth_chroma_inplace(v, (size_t)frames, (size_t)window);
    } else if (frames > 0 && window > 1) {
        const int64_t half = (int64_t)window / 2;
        std::vector<float> o(v.size());
        for (int64_t t = 0; t < (int64_t)frames; t++)
            for (int s = 0; s < 12; s++) {
                float sum = 0.0f;
                int cnt = 0;
                for (int64_t k = 0; k < (int64_t)window; k++) {
                    const int64_t fi = t + (k - half);
                    if (fi >= 0 && fi < (int64_t)frames) {
                        sum += v[(size_t)fi * 12 + (size_t)s];
                        cnt++;
                    }
                }
                o[(size_t)t * 12 + (size_t)s] = cnt > 0 ? sum / (float)cnt : v[(size_t)t * 12 + (size_t)s];
            }
        v.swap(o);
    }
    std::memcpy(out, v.data(), v.size() * sizeof(float));
}

// dot_product (detector.rs:979-981): sequential f32 sum of products
float sdsp_oracle_dot(const float* a, const float* b, uint64_t n) {
    float acc = 0.0f;
    for (uint64_t i = 0; i < n; i++) acc += a[i] * b[i];
    return acc;
}
}

// study switches (oracle_internal.hpp): not used by the parity tests
extern "C" void sdsp_oracle_study_block_energy(int32_t on) { orc::g_block_energy = on; }
extern "C" void sdsp_oracle_study_key_trace(int32_t on) {
    static std::vector<float> tr;
    tr.clear();
    orc::g_key_trace = on ? &tr : nullptr;
}
extern "C" uint64_t sdsp_oracle_study_key_trace_get(float* out, uint64_t cap) {
    if (!orc::g_key_trace) return 0;
    const uint64_t n = orc::g_key_trace->size();
    for (uint64_t i = 0; i < n && i < cap; i++) out[i] = (*orc::g_key_trace)[(size_t)i];
    return n;
}
