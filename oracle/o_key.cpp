// o_key.cpp — key path (TEST INFRASTRUCTURE, see oracle_internal.hpp).
//
// Follows src/features/chroma/extractor.rs:529-680 (HPCP), :1097-1150 (driver + energies),
// :1246-1349 (time smoothing + harmonic mask); src/features/chroma/smoothing.rs:37-94;
// src/features/key/{detector.rs:68-313,984-1001; templates.rs:64-145; key_clarity.rs:51-93}.
#include <algorithm>

#include "oracle_internal.hpp"

namespace orc {

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

// templates.rs:64-145 (K-K profiles rotated, then L2-normalised per key in rotated order)
void key_templates(float maj[12][12], float min_[12][12]) {
    const float cM[12] = {6.35f, 2.23f, 3.48f, 2.33f, 4.38f, 4.09f, 2.52f, 5.19f, 2.39f, 3.66f, 2.29f, 2.88f};
    const float cm[12] = {6.33f, 2.68f, 3.52f, 5.38f, 2.60f, 3.53f, 2.54f, 4.75f, 3.98f, 2.69f, 3.34f, 3.17f};
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
