// o_chroma.cpp — the key path's opt-in chroma front-ends (TEST INFRASTRUCTURE, see
// oracle_internal.hpp).
//
// Follows src/features/chroma/extractor.rs:
//   :66-177    estimate_tuning_offset_semitones_from_spectrogram
//   :393-481   frame_to_chroma_tuned (+ :1028-1094 the per-frame energies)
//   :529-680   frame_to_hpcp_tuned_band with tuning, whitening and any band
//   :1097-1244 the HPCP and HPCP bass-blend drivers
//   :701-828   convert_linear_to_log_frequency_spectrogram, :937-985 its chroma
//   :830-935   extract_beat_synchronous_chroma
//   :1246-1290 smooth_spectrogram_time (time smoothing without the harmonic mask)
// and the dispatch at src/lib.rs:1063-1198.
#include <algorithm>

#include "oracle_internal.hpp"

namespace orc {

namespace {

constexpr float A4 = 440.0f, SEMI0 = 57.0f;
constexpr float CHROMA_FMIN = 100.0f, CHROMA_FMAX = 5000.0f;
constexpr float TWO_PI_F = 2.0f * 3.14159265358979323846f;  // 2.0 * std::f32::consts::PI

// compiler-rt __powisf2 (Rust f32::powi with a runtime exponent)
float powi_f(float a, int b) {
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

// circular soft mapping of one contribution onto 3 pitch classes (extractor.rs:437-455, :653-667)
void soft_map(float* pc, float semitone, float contrib, float sigma_in) {
    const float spc = sd_rem_euclid_f(semitone, 12.0f);
    const float ppc = sd_rem_euclid_f(sd_roundf(spc), 12.0f);
    const int32_t primary = sd_f2i32(ppc);
    for (int off = -1; off <= 1; off++) {
        const int tc = (((primary + off) % 12) + 12) % 12;
        float dist = sd_absf(spc - (float)tc);
        dist = sd_minf(dist, 12.0f - dist);
        const float sigma = sd_maxf(sigma_in, 1e-6f);
        pc[tc] += contrib * sd_expf(-dist * dist / (2.0f * sigma * sigma));
    }
}

void l2_normalize(float* pc, float eps) {
    float nsq = 0.0f;
    for (int i = 0; i < 12; i++) nsq += pc[i] * pc[i];
    const float norm = __builtin_sqrtf(nsq);
    if (norm > eps)
        for (int i = 0; i < 12; i++) pc[i] /= norm;
}

float frame_energy(const float* m, size_t bins) {
    float e = 0.0f;
    if (g_block_energy) {  // the GPU's block order: 64-bin partial sums, then those in block order
        for (size_t g = 0; g < bins; g += 64) {
            float p = 0.0f;
            for (size_t b = g; b < g + 64 && b < bins; b++) p += m[b] * m[b];
            e += p;
        }
        return e;
    }
    for (size_t b = 0; b < bins; b++) e += m[b] * m[b];
    return e;
}

}  // namespace

// extractor.rs:66-177
float estimate_tuning(const Spec& s, uint32_t sr, size_t fft_size, float fmin_hz, float fmax_hz, size_t frame_step,
                      float peak_rel_threshold) {
    if (s.empty() || sr == 0 || fft_size == 0) return 0.0f;
    const float fres = (float)sr / (float)fft_size;
    const float fmin = sd_maxf(fmin_hz, 20.0f);
    const float fmax = sd_clampf(fmax_hz, fmin + 1.0f, (float)sr / 2.0f);
    const size_t step = std::max<size_t>(frame_step, 1);
    const float thr = sd_clampf(peak_rel_threshold, 0.0f, 1.0f);
    float ss = 0.0f, sc = 0.0f, sw = 0.0f;
    for (size_t t = 0; t < s.frames; t += step) {
        const float* m = s.row(t);
        float peak = 0.0f;
        for (size_t b = 0; b < s.bins; b++) {
            const float f = (float)b * fres;
            if (f < fmin) continue;
            if (f > fmax) break;
            peak = sd_maxf(peak, m[b]);
        }
        if (peak <= 1e-12f) continue;
        const float abs_thr = peak * thr;
        for (size_t b = 0; b < s.bins; b++) {
            if (m[b] < abs_thr) continue;
            const float f = (float)b * fres;
            if (f < fmin) continue;
            if (f > fmax) break;
            const float semitone = 12.0f * sd_log2f(f / A4) + SEMI0;
            const float residual = semitone - sd_roundf(semitone);
            const float w = sd_powf(sd_maxf(m[b], 0.0f), 0.5f);
            if (w <= 0.0f) continue;
            const float angle = TWO_PI_F * residual;
            ss += w * sd_sinf(angle);
            sc += w * sd_cosf(angle);
            sw += w;
        }
    }
    if (sw <= 1e-6f) return 0.0f;
    const float r = __builtin_sqrtf(ss * ss + sc * sc) / sw;
    if (r < 0.05f) return 0.0f;
    return sd_atan2f(ss, sc) / TWO_PI_F;
}

// extractor.rs:393-481 (frame_to_chroma_tuned) for every frame, with :1080-1090's energies
void chroma_frames(const Spec& s, uint32_t sr, size_t fft_size, bool soft, float sigma, float tuning,
                   std::vector<float>* chroma12, std::vector<float>* energies) {
    chroma12->assign(s.frames * 12, 0.0f);
    energies->assign(s.frames, 0.0f);
    const float fres = (float)sr / (float)fft_size;
    const float nyq = (float)sr / 2.0f;
    const float hi = sd_minf(CHROMA_FMAX, nyq);
    for (size_t t = 0; t < s.frames; t++) {
        const float* m = s.row(t);
        (*energies)[t] = frame_energy(m, s.bins);
        float* pc = chroma12->data() + t * 12;
        for (size_t b = 0; b < s.bins; b++) {
            const float f = (float)b * fres;
            if (f < CHROMA_FMIN) continue;
            if (f > hi) break;
            if (f >= nyq) break;
            const float semitone = 12.0f * sd_log2f(f / A4) + SEMI0 - tuning;
            const float mag = sd_powf(sd_maxf(m[b], 0.0f), 0.6f);
            if (soft) {
                soft_map(pc, semitone, mag, sigma);
            } else {
                int32_t cls = sd_f2i32(sd_roundf(semitone)) % 12;
                if (cls < 0) cls += 12;
                pc[cls] += mag;
            }
        }
        l2_normalize(pc, EPS);
    }
}

// extractor.rs:529-680 for one frame: tuning, optional whitening, band [fmin_hz, fmax_hz].
// Top-K peaks in (score desc, bin asc) order (select_nth_unstable_by's order is
// implementation-defined in the reference).
static void hpcp_frame_band(const float* m, size_t bins, uint32_t sr, size_t fft_size, const HpcpCfg& c,
                            size_t peaks_k, float fmin_hz, float fmax_hz, float* pc, std::vector<float>& white,
                            std::vector<float>& prefix, std::vector<std::pair<size_t, float>>& peaks) {
    for (int i = 0; i < 12; i++) pc[i] = 0.0f;
    if (bins == 0 || sr == 0 || fft_size == 0) return;
    const float fres = (float)sr / (float)fft_size;
    const float fmin = sd_maxf(fmin_hz, 20.0f);
    const float fmax = sd_minf(fmax_hz, (float)sr / 2.0f);
    if (fmax <= fmin) return;
    const bool wh = c.whitening && c.whitening_bins >= 3;
    if (wh) {
        const size_t win = std::max<size_t>(c.whitening_bins, 3) | 1;
        const size_t half = win / 2;
        prefix.assign(bins + 1, 0.0f);
        for (size_t i = 0; i < bins; i++) prefix[i + 1] = prefix[i] + sd_maxf(m[i], 0.0f);
        white.assign(bins, 0.0f);
        for (size_t i = 0; i < bins; i++) {
            const size_t l = i >= half ? i - half : 0;
            const size_t r = std::min(i + half, bins - 1);
            const float denom = (float)(r + 1 - l);
            const float mean = (prefix[r + 1] - prefix[l]) / sd_maxf(denom, 1.0f);
            const float v = sd_maxf(m[i], 0.0f) / (mean + 1e-12f);
            white[i] = sd_minf(v, 20.0f);
        }
    }
    const float* sc = wh ? white.data() : m;
    peaks.clear();
    for (size_t bin = 1; bin + 1 < bins; bin++) {
        const float f = (float)bin * fres;
        if (f < fmin) continue;
        if (f > fmax) break;
        const float mv = sc[bin], mp = sc[bin - 1], mn = sc[bin + 1];
        if (mv <= mp || mv < mn) continue;
        // A NaN score (a NaN magnitude: non-finite input) passes the reference's local-maximum
        // test, and its rank is then implementation-defined (select_nth_unstable_by with
        // partial_cmp -> Equal: parity unpinned).  The restatement, like the kernels, ranks NaN
        // below every peak, i.e. never selects it (its weight powf(max(NaN, 0), p) would be 0).
        if (mv != mv) continue;
        peaks.push_back({bin, mv});
    }
    if (peaks.empty()) return;
    const size_t k = std::min(std::max<size_t>(peaks_k, 1), peaks.size());
    std::stable_sort(peaks.begin(), peaks.end(), [](auto& a, auto& b) { return b.second < a.second; });
    peaks.resize(k);
    const size_t hmax = std::max<size_t>(c.harmonics, 1);
    const float decay = sd_clampf(c.decay, 0.0f, 1.0f);
    const float p = sd_clampf(c.mag_power, 0.05f, 1.0f);
    for (auto& pk : peaks) {
        const float f0 = (float)pk.first * fres;
        if (f0 <= 0.0f) continue;
        const float w0 = sd_powf(sd_maxf(m[pk.first], 0.0f), p);
        if (w0 <= 0.0f) continue;
        for (size_t h = 1; h <= hmax; h++) {
            const float fh = f0 * (float)h;
            if (fh > fmax) break;
            if (fh < fmin) continue;
            const float semitone = 12.0f * sd_log2f(fh / A4) + SEMI0 - c.tuning;
            const float hw = powi_f(decay, (int)h - 1) / (float)h;
            soft_map(pc, semitone, w0 * hw, c.sigma);
        }
    }
    l2_normalize(pc, EPS);
}

// extractor.rs:1097-1150 (bass_blend false) and :1154-1244 (bass_blend true)
void hpcp_frames_x(const Spec& s, uint32_t sr, size_t fft_size, const HpcpCfg& c, std::vector<float>* chroma12,
                   std::vector<float>* energies) {
    chroma12->assign(s.frames * 12, 0.0f);
    energies->assign(s.frames, 0.0f);
    std::vector<float> white, prefix;
    std::vector<std::pair<size_t, float>> peaks;
    const float w = sd_clampf(c.bass_weight, 0.0f, 1.0f);
    for (size_t t = 0; t < s.frames; t++) {
        const float* m = s.row(t);
        (*energies)[t] = frame_energy(m, s.bins);
        float* pc = chroma12->data() + t * 12;
        hpcp_frame_band(m, s.bins, sr, fft_size, c, c.peaks, CHROMA_FMIN, CHROMA_FMAX, pc, white, prefix, peaks);
        if (!c.bass_blend) continue;
        float bass[12];
        hpcp_frame_band(m, s.bins, sr, fft_size, c, std::min<size_t>(std::max<size_t>(c.peaks, 1), 12), c.bass_fmin,
                        c.bass_fmax, bass, white, prefix, peaks);
        for (int i = 0; i < 12; i++) pc[i] = (1.0f - w) * pc[i] + w * bass[i];
        l2_normalize(pc, 1e-10f);
    }
}

// extractor.rs:701-828 + :937-985, energies per src/lib.rs:1120-1131.  Returns false when the
// semitone range is degenerate (the reference would fail to allocate; never for sr >= 10.2 kHz).
bool log_freq_chroma(const Spec& s, uint32_t sr, size_t fft_size, std::vector<float>* chroma12,
                     std::vector<float>* energies) {
    const float fres = (float)sr / (float)fft_size;
    const float nyq = (float)sr / 2.0f;
    const float fmin = sd_maxf(CHROMA_FMIN, 20.0f);
    const float fmax = sd_minf(CHROMA_FMAX, nyq - 1.0f);
    const float smin = 12.0f * sd_log2f(fmin / A4) + SEMI0;
    const float smax = 12.0f * sd_log2f(fmax / A4) + SEMI0;
    const int32_t bmin = sd_f2i32(__builtin_floorf(smin));
    const int32_t bmax = sd_f2i32(__builtin_ceilf(smax));
    if (bmax - bmin + 1 <= 0) return false;
    const size_t n = (size_t)(bmax - bmin + 1);
    chroma12->assign(s.frames * 12, 0.0f);
    energies->assign(s.frames, 0.0f);
    std::vector<float> lf(n);
    // semitone offset of the first bin (src/lib.rs:1074-1077: the same floor with fmin = 100)
    const int32_t off = sd_f2i32(__builtin_floorf(12.0f * sd_log2f(100.0f / A4) + SEMI0));
    for (size_t t = 0; t < s.frames; t++) {
        const float* m = s.row(t);
        std::fill(lf.begin(), lf.end(), 0.0f);
        for (size_t b = 0; b < s.bins; b++) {
            const float mag = m[b];
            if (mag <= 0.0f) continue;
            const float f = (float)b * fres;
            if (f < fmin || f >= fmax || f >= nyq) continue;
            const float semitone = 12.0f * sd_log2f(f / A4) + SEMI0;
            const float sf = semitone - (float)bmin;
            const size_t lo = (size_t)sd_f2u64(__builtin_floorf(sf));
            const size_t hi = std::min<size_t>((size_t)sd_f2u64(__builtin_ceilf(sf)), n - 1);
            if (lo < n) {
                const float wh = sf - (float)lo;
                const float wl = 1.0f - wh;
                lf[lo] += mag * wl;
                if (hi != lo && hi < n) lf[hi] += mag * wh;
            }
        }
        float* pc = chroma12->data() + t * 12;
        for (size_t b = 0; b < n; b++) {
            if (lf[b] <= 0.0f) continue;
            int32_t cls = (off + (int32_t)b) % 12;
            if (cls < 0) cls += 12;
            pc[cls] += lf[b];
        }
        l2_normalize(pc, EPS);
        float e = 0.0f;
        for (size_t b = 0; b < n; b++) e += lf[b] * lf[b];
        (*energies)[t] = e;
    }
    return true;
}

// extractor.rs:830-935: one chroma row per beat interval [beats[i], beats[i+1]).  Frame chroma
// is frame_to_chroma_tuned (computed once per frame: it is a pure function of the frame).
void beat_sync_chroma(const Spec& s, uint32_t sr, size_t fft_size, size_t hop, const std::vector<float>& beats,
                      bool soft, float sigma, float tuning, std::vector<float>* chroma12, std::vector<float>* energies) {
    chroma12->clear();
    energies->clear();
    if (s.empty() || beats.size() < 2) return;
    std::vector<float> fc, fe;
    chroma_frames(s, sr, fft_size, soft, sigma, tuning, &fc, &fe);
    const float fd = (float)hop / (float)sr;
    const size_t NB = beats.size() - 1;
    chroma12->assign(NB * 12, 0.0f);
    energies->assign(NB, 0.0f);
    for (size_t i = 0; i < NB; i++) {
        const float bs = beats[i], be = beats[i + 1];
        float avg[12] = {0};
        float e = 0.0f;
        size_t cnt = 0;
        for (size_t f = 0; f < s.frames; f++) {
            const float ft = (float)f * fd;
            if (ft >= bs && ft < be) {
                for (int j = 0; j < 12; j++) avg[j] += fc[f * 12 + j];
                e += fe[f];
                cnt++;
            }
        }
        if (cnt == 0) continue;
        const float nf = (float)cnt;
        for (int j = 0; j < 12; j++) avg[j] /= nf;
        l2_normalize(avg, EPS);
        std::copy(avg, avg + 12, chroma12->data() + i * 12);
        (*energies)[i] = e;
    }
}

// extractor.rs:1246-1290 (margin 0 returns the input)
void smooth_time_inplace(Spec& s, size_t margin) {
    if (s.empty() || margin == 0) return;
    const size_t F = s.frames, B = s.bins;
    std::vector<float> pre(F + 1), out(F);
    for (size_t b = 0; b < B; b++) {
        pre[0] = 0.0f;
        for (size_t t = 0; t < F; t++) pre[t + 1] = pre[t] + s.row(t)[b];
        for (size_t t = 0; t < F; t++) {
            const size_t st = t >= margin ? t - margin : 0;
            const size_t en = std::min(t + margin + 1, F);
            out[t] = (pre[en] - pre[st]) / (float)std::max<size_t>(en - st, 1);
        }
        for (size_t t = 0; t < F; t++) s.row(t)[b] = out[t];
    }
}

}  // namespace orc

// ---- probes for tests/test_oracle_chroma.py ----
extern "C" {

// mode 0 frame_to_chroma_tuned, 1 HPCP (default options + tuning), 2 log-frequency chroma,
// 3 beat-synchronous chroma.  Returns the number of chroma rows written (<= cap), or -1.
int64_t sdsp_oracle_chroma(int32_t mode, const float* spec, uint64_t frames, uint64_t bins, uint32_t sr,
                           uint64_t fft_size, uint64_t hop, int32_t soft, float sigma, float tuning, const float* beats,
                           uint64_t n_beats, float* out_chroma, float* out_energy, uint64_t cap) {
    using namespace orc;
    Spec s;
    s.frames = (size_t)frames;
    s.bins = (size_t)bins;
    s.d.assign(spec, spec + frames * bins);
    std::vector<float> ch, en;
    if (mode == 0) {
        chroma_frames(s, sr, (size_t)fft_size, soft != 0, sigma, tuning, &ch, &en);
    } else if (mode == 1) {
        HpcpCfg c;
        c.sigma = sigma;
        c.tuning = tuning;
        hpcp_frames_x(s, sr, (size_t)fft_size, c, &ch, &en);
    } else if (mode == 2) {
        if (!log_freq_chroma(s, sr, (size_t)fft_size, &ch, &en)) return -1;
    } else {
        std::vector<float> b(beats, beats + n_beats);
        beat_sync_chroma(s, sr, (size_t)fft_size, (size_t)hop, b, soft != 0, sigma, tuning, &ch, &en);
    }
    const uint64_t rows = en.size();
    if (rows > cap) return -1;
    std::copy(ch.begin(), ch.end(), out_chroma);
    std::copy(en.begin(), en.end(), out_energy);
    return (int64_t)rows;
}

float sdsp_oracle_tuning(const float* spec, uint64_t frames, uint64_t bins, uint32_t sr, uint64_t fft_size,
                         uint64_t frame_step, float rel_threshold) {
    using namespace orc;
    Spec s;
    s.frames = (size_t)frames;
    s.bins = (size_t)bins;
    s.d.assign(spec, spec + frames * bins);
    return estimate_tuning(s, sr, (size_t)fft_size, 80.0f, 2000.0f, (size_t)frame_step, rel_threshold);
}

}  // extern "C"

namespace orc {

// extractor.rs:1369-1501 (harmonic_spectrogram_hpss_median_mask), in place.  The medians are
// order statistics (element len/2 of the sorted window), so any selection algorithm gives the
// reference's value.
void key_hpss_mask_inplace(Spec& s, uint32_t sr, size_t fft_size, float fmin_hz, float fmax_hz, size_t frame_step,
                           size_t time_margin, size_t freq_margin, float mask_power) {
    if (s.empty() || sr == 0 || fft_size == 0) return;
    const size_t F = s.frames, B = s.bins;
    const float fres = (float)sr / (float)fft_size;
    const float fmin = sd_maxf(fmin_hz, 20.0f);
    const float fmax = sd_clampf(fmax_hz, fmin + 1.0f, (float)sr / 2.0f);
    int64_t bs = sd_f2i64(__builtin_floorf(fmin / fres)), be = sd_f2i64(__builtin_ceilf(fmax / fres));
    bs = std::min<int64_t>(std::max<int64_t>(bs, 0), (int64_t)B);
    be = std::min<int64_t>(std::max<int64_t>(be, 0), (int64_t)B);
    if (be <= bs) return;
    const size_t b0 = (size_t)bs, nb = (size_t)(be - bs);
    const size_t step = std::max<size_t>(frame_step, 1);
    const size_t nds = std::max<size_t>((F + step - 1) / step, 1);
    auto san = [](float x) { return sd_isfinite_f(x) ? sd_maxf(x, 0.0f) : 0.0f; };
    std::vector<float> ds(nds * nb), h(nds * nb), pe(nds * nb);
    for (size_t k = 0; k < nds; k++)
        for (size_t b = 0; b < nb; b++) ds[k * nb + b] = s.row(k * step)[b0 + b];
    std::vector<float> w;
    auto median = [&](std::vector<float>& v) {
        if (v.empty()) return 0.0f;
        const size_t mid = v.size() / 2;
        std::nth_element(v.begin(), v.begin() + (long)mid, v.end());
        return v[mid];
    };
    for (size_t b = 0; b < nb; b++)
        for (size_t t = 0; t < nds; t++) {
            w.clear();
            const size_t st = t >= time_margin ? t - time_margin : 0, en = std::min(t + time_margin + 1, nds);
            for (size_t k = st; k < en; k++) w.push_back(san(ds[k * nb + b]));
            h[t * nb + b] = median(w);
        }
    for (size_t t = 0; t < nds; t++)
        for (size_t b = 0; b < nb; b++) {
            w.clear();
            const size_t st = b >= freq_margin ? b - freq_margin : 0, en = std::min(b + freq_margin + 1, nb);
            for (size_t q = st; q < en; q++) w.push_back(san(ds[t * nb + q]));
            pe[t * nb + b] = median(w);
        }
    const float p = sd_maxf(mask_power, 1.0f);
    std::vector<float> mask(nds * nb);
    for (size_t i = 0; i < nds * nb; i++) {
        const float hh = sd_maxf(h[i], 0.0f), pp = sd_maxf(pe[i], 0.0f);
        const float hp = sd_powf(hh, p), ppw = sd_powf(pp, p);
        mask[i] = hp / (hp + ppw + 1e-12f);
    }
    for (size_t t = 0; t < F; t++) {
        float* row = s.row(t);
        const size_t k = std::min(t / step, nds - 1);
        for (size_t b = 0; b < B; b++) {
            if (b < b0 || b >= b0 + nb) {
                row[b] = 0.0f;  // the reference's output starts as zeros; only the band is written
                continue;
            }
            row[b] = san(row[b]) * mask[k * nb + (b - b0)];
        }
    }
}

}  // namespace orc

extern "C" void sdsp_oracle_key_hpss(float* spec, uint64_t frames, uint64_t bins, uint32_t sr, uint64_t fft_size,
                                     uint64_t step, uint64_t tm, uint64_t fm, float power) {
    orc::Spec s;
    s.frames = (size_t)frames;
    s.bins = (size_t)bins;
    s.d.assign(spec, spec + frames * bins);
    orc::key_hpss_mask_inplace(s, sr, (size_t)fft_size, 100.0f, 5000.0f, (size_t)step, (size_t)tm, (size_t)fm, power);
    std::copy(s.d.begin(), s.d.end(), spec);
}
