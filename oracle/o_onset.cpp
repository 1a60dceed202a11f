// o_onset.cpp — preprocessing and onset detectors (TEST INFRASTRUCTURE, see oracle_internal.hpp).
#include <algorithm>
#include <cmath>

#include "oracle_internal.hpp"

namespace orc {

// src/preprocessing/normalization.rs:262-322 (normalize_peak; the RMS it computes is metadata only)
void normalize_peak(std::vector<float>& x, float headroom_db) {
    if (x.empty()) fail(SDSP_ERR_INVALID_INPUT, "Empty audio samples");
    float peak = 0.0f;
    for (float v : x) peak = sd_maxf(peak, sd_absf(v));  // fold(0.0, f32::max)
    if (peak <= EPS) return;                               // :276-284
    const float target = sd_powf(10.0f, (0.0f - headroom_db) / 20.0f);
    float gain = target / peak;
    gain = sd_minf(gain, 1.0f / peak);  // :296
    for (float& v : x) v *= gain;
}

// normalization.rs:325-402 (normalize_rms; target_rms_db = target_lufs + 3, :534-539)
void normalize_rms(std::vector<float>& x, float target_lufs, float headroom_db) {
    if (x.empty()) fail(SDSP_ERR_INVALID_INPUT, "Empty audio samples");
    float ss = 0.0f;
    for (float v : x) ss += v * v;
    const float rms = std::sqrt(ss / (float)x.size());
    if (rms <= EPS) return;
    float peak = 0.0f;
    for (float v : x) peak = sd_maxf(peak, sd_absf(v));
    const float target_rms_db = target_lufs + 3.0f;
    const float target = sd_powf(10.0f, (target_rms_db - headroom_db) / 20.0f);
    float gain = target / rms;
    if (peak * gain > 1.0f) gain = 1.0f / peak;  // :367-385
    for (float& v : x) v *= gain;
}

// normalization.rs:119-158 (KWeightingFilter) and :183-259 (calculate_lufs); returns false for
// the -inf case (every block below the gate)
static bool calculate_lufs(const std::vector<float>& x, uint32_t sr, float* lufs) {
    const float fsr = (float)sr;
    const size_t block = sd_f2u64(fsr * 400.0f / 1000.0f);
    if (block == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate too low for LUFS calculation");
    const float w0 = 2.0f * 3.14159274f * 1681.9745f / fsr;
    const float cw = std::cos(w0), sw = std::sin(w0);
    const float alpha = sw / 2.0f * std::sqrt(1.0f / 0.707f);
    const float a0 = 1.0f + alpha;
    const float b0 = ((1.0f + cw) / 2.0f) / a0, b1 = (-(1.0f + cw)) / a0, b2 = ((1.0f + cw) / 2.0f) / a0;
    const float a1 = (-2.0f * cw) / a0, a2 = (1.0f - alpha) / a0;
    float x1 = 0.0f, x2 = 0.0f;
    std::vector<float> y(x.size());
    for (size_t i = 0; i < x.size(); i++) {  // Direct Form II transposed
        const float s = x[i];
        const float o = b0 * s + x1;
        x1 = b1 * s + x2 - a1 * o;
        x2 = b2 * s - a2 * o;
        y[i] = o;
    }
    const float gate = sd_powf(10.0f, (-70.0f + 0.691f) / 10.0f);
    float gsum = 0.0f;
    size_t gn = 0;
    for (size_t st = 0; st < y.size(); st += block) {
        const size_t en = std::min(st + block, y.size());
        float sq = 0.0f;
        for (size_t i = st; i < en; i++) sq += y[i] * y[i];
        const float ms = sq / (float)(en - st);
        if (ms > gate) {
            gsum += ms;
            gn++;
        }
    }
    if (gn == 0) return false;
    const float mean = gsum / (float)gn;
    if (mean <= EPS) fail(SDSP_ERR_NUMERICAL, "Mean square too small for LUFS calculation");
    *lufs = -0.691f + 10.0f * sd_log10f(mean);
    return true;
}

// normalization.rs:405-470 (normalize_lufs)
void normalize_lufs(std::vector<float>& x, uint32_t sr, float target_lufs, float headroom_db) {
    if (x.empty()) fail(SDSP_ERR_INVALID_INPUT, "Empty audio samples");
    float lufs;
    if (!calculate_lufs(x, sr, &lufs)) {
        normalize_peak(x, headroom_db);
        return;
    }
    const float gain = sd_powf(10.0f, (target_lufs - lufs) / 20.0f);
    float peak = 0.0f;
    for (float v : x) peak = sd_maxf(peak, sd_absf(v));
    const float tpl = sd_powf(10.0f, (0.0f - headroom_db) / 20.0f);
    const float g = peak * gain > tpl ? tpl / peak : gain;
    for (float& v : x) v *= g;
}

// src/preprocessing/silence.rs:102-279
void detect_and_trim(const std::vector<float>& x, uint32_t sr, float threshold_db, uint32_t min_ms,
                     size_t frame_size, size_t* trim_start, size_t* trim_end,
                     std::vector<std::pair<size_t, size_t>>* silence_map) {
    const size_t n = x.size();
    if (silence_map) silence_map->clear();
    if (n == 0) {
        *trim_start = *trim_end = 0;
        return;
    }
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate must be > 0");
    if (frame_size == 0) fail(SDSP_ERR_INVALID_INPUT, "Frame size must be > 0");
    const float thr = sd_powf(10.0f, threshold_db / 20.0f);
    const size_t hop = frame_size / 2;
    const size_t num_frames = n >= frame_size ? (n - frame_size) / hop + 1 : 1;
    std::vector<char> silent(num_frames);
    std::vector<size_t> starts(num_frames);
    for (size_t i = 0; i < num_frames; i++) {
        const size_t s = i * hop, e = std::min(s + frame_size, n);
        float sum = 0.0f;
        for (size_t k = s; k < e; k++) sum += x[k] * x[k];
        const float rms = e > s ? __builtin_sqrtf(sum / (float)(e - s)) : 0.0f;
        silent[i] = rms <= thr;
        starts[i] = s;
    }
    const size_t min_samples = (size_t)sd_f2u64((float)min_ms / 1000.0f * (float)sr);
    const size_t min_frames = (min_samples + hop - 1) / hop;  // div_ceil
    struct R {
        size_t s, e;
    };
    std::vector<R> regions;
    bool in_sil = false;
    size_t sil_start = 0;
    for (size_t f = 0; f < num_frames; f++) {
        if (silent[f] && !in_sil) {
            in_sil = true;
            sil_start = f;
        } else if (!silent[f] && in_sil) {
            in_sil = false;
            const size_t end_f = f;
            if (end_f - sil_start >= min_frames || sil_start == 0 || end_f == num_frames) {
                const size_t ss = starts[sil_start];
                const size_t es = end_f < starts.size() ? starts[end_f] : n;
                regions.push_back({ss, es});
            }
        }
    }
    if (in_sil) {
        if (num_frames - sil_start >= min_frames || sil_start == 0) regions.push_back({starts[sil_start], n});
    }
    if (silence_map)
        for (auto& r : regions) silence_map->push_back({r.s, r.e});
    size_t ts = 0, te = n;
    if (!regions.empty() && regions.front().s == 0) ts = regions.front().e;
    if (!regions.empty() && regions.back().e == n) te = regions.back().s;
    ts = std::min(ts, te);
    te = std::max(te, ts);
    if (!(ts < te && te <= n)) ts = te = 0;
    *trim_start = ts;
    *trim_end = te;
}

// src/features/onset/energy_flux.rs:60-243
std::vector<size_t> energy_flux_onsets(const float* s, size_t n, size_t frame, size_t hop, float thr_db) {
    std::vector<size_t> on;
    if (n == 0) return on;
    if (frame == 0) fail(SDSP_ERR_INVALID_INPUT, "Frame size must be > 0");
    if (hop == 0) fail(SDSP_ERR_INVALID_INPUT, "Hop size must be > 0");
    if (frame > n) return on;
    const size_t nf = (n - frame) / hop + 1;
    if (nf < 2) return on;
    std::vector<float> e(nf);
    for (size_t i = 0; i < nf; i++) {
        const size_t st = i * hop, en = std::min(st + frame, n);
        float sum = 0.0f;
        for (size_t k = st; k < en; k++) sum += s[k] * s[k];
        e[i] = __builtin_sqrtf(sum / (float)(en - st));
    }
    std::vector<float> flux(nf - 1);
    for (size_t i = 1; i < nf; i++) flux[i - 1] = sd_maxf(e[i] - e[i - 1], 0.0f);
    float mx = 0.0f;
    for (float v : flux) mx = sd_maxf(mx, v);
    if (mx <= EPS) return on;
    const float thr = mx * sd_powf(10.0f, thr_db / 20.0f);
    const size_t L = flux.size();
    for (size_t i = 1; i + 1 < L; i++) {
        const float f = flux[i];
        if (f > thr && f > flux[i - 1] && f >= flux[i + 1]) {
            const size_t o = (i + 1) * hop;
            if (o < n) on.push_back(o);
        }
    }
    if (L > 1 && flux[0] > thr && flux[0] >= flux[1]) {
        if (hop < n) on.push_back(hop);
    }
    const size_t li = L - 1;
    if (L > 1 && flux[li] > thr && flux[li] > flux[li - 1]) {
        const size_t o = (li + 1) * hop;
        if (o < n) on.push_back(o);
    }
    std::sort(on.begin(), on.end());
    if (!on.empty()) {
        std::vector<size_t> d{on[0]};
        for (size_t k = 1; k < on.size(); k++)
            if (on[k] >= d.back() + hop / 2) d.push_back(on[k]);
        on.swap(d);
    }
    return on;
}

// Shared tail of spectral_flux.rs:165-215 and hfc.rs:162-208: percentile threshold + peaks.
static std::vector<size_t> peaks_over_percentile(const std::vector<float>& flux, float pct) {
    std::vector<size_t> on;
    if (flux.empty()) return on;
    std::vector<float> sorted(flux);
    std::stable_sort(sorted.begin(), sorted.end(), [](float a, float b) { return a < b; });
    size_t ti = (size_t)sd_f2u64((float)sorted.size() * pct);
    ti = std::min(ti, sorted.size() - 1);
    const float thr = sorted[ti];
    const size_t L = flux.size();
    for (size_t i = 1; i + 1 < L; i++) {
        const float f = flux[i];
        if (f > thr && f > flux[i - 1] && f >= flux[i + 1]) on.push_back(i + 1);
    }
    if (L > 1 && flux[0] > thr && flux[0] >= flux[1]) on.push_back(1);
    const size_t li = L - 1;
    if (L > 1 && flux[li] > thr && flux[li] > flux[li - 1]) on.push_back(L);
    std::sort(on.begin(), on.end());
    on.erase(std::unique(on.begin(), on.end()), on.end());
    return on;
}

// src/features/onset/spectral_flux.rs:60-221
std::vector<size_t> spectral_flux_onsets(const Spec& m, float pct) {
    if (m.empty()) return {};
    if (!(pct >= 0.0f && pct <= 1.0f)) fail(SDSP_ERR_INVALID_INPUT, "Threshold percentile must be in [0, 1]");
    if (m.bins == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty magnitude frames");
    if (m.frames < 2) return {};
    const size_t B = m.bins;
    std::vector<float> mx(m.frames);
    for (size_t t = 0; t < m.frames; t++) {
        float v = 0.0f;
        const float* r = m.row(t);
        for (size_t b = 0; b < B; b++) v = sd_maxf(v, r[b]);
        mx[t] = v;
    }
    std::vector<float> flux(m.frames - 1);
    for (size_t t = 1; t < m.frames; t++) {
        const float* p = m.row(t - 1);
        const float* c = m.row(t);
        const bool pn = mx[t - 1] > EPS, cn = mx[t] > EPS;
        float sum = 0.0f;
        for (size_t b = 0; b < B; b++) {
            const float pv = pn ? p[b] / mx[t - 1] : 0.0f;
            const float cv = cn ? c[b] / mx[t] : 0.0f;
            const float d = sd_maxf(cv - pv, 0.0f);
            sum += d * d;
        }
        flux[t - 1] = __builtin_sqrtf(sum);
    }
    return peaks_over_percentile(flux, pct);
}

// src/features/onset/hfc.rs:70-214
std::vector<size_t> hfc_onsets(const Spec& m, uint32_t sr, float pct) {
    if (m.empty()) return {};
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate must be > 0");
    if (!(pct >= 0.0f && pct <= 1.0f)) fail(SDSP_ERR_INVALID_INPUT, "Threshold percentile must be in [0, 1]");
    if (m.bins == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty magnitude frames");
    if (m.frames < 2) return {};
    std::vector<float> h(m.frames);
    for (size_t t = 0; t < m.frames; t++) {
        const float* r = m.row(t);
        float acc = 0.0f;
        for (size_t b = 0; b < m.bins; b++) acc += (float)b * r[b] * r[b];
        h[t] = acc;
    }
    std::vector<float> flux(m.frames - 1);
    for (size_t t = 1; t < m.frames; t++) flux[t - 1] = sd_maxf(h[t] - h[t - 1], 0.0f);
    return peaks_over_percentile(flux, pct);
}

// src/features/onset/consensus.rs:111-287
std::vector<OnsetCand> vote_onsets(const std::vector<size_t> lists[4], const float w[4], uint32_t tol_ms,
                                   uint32_t sr) {
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate must be > 0");
    if (tol_ms == 0) fail(SDSP_ERR_INVALID_INPUT, "Tolerance must be > 0");
    for (int i = 0; i < 4; i++)
        if (w[i] < 0.0f) fail(SDSP_ERR_INVALID_INPUT, "Weights must be non-negative");
    const size_t tol = (size_t)sd_f2u64((float)tol_ms / 1000.0f * (float)sr);
    struct O {
        size_t sample;
        int method;
        float weight;
    };
    std::vector<O> all;
    for (int mth = 0; mth < 4; mth++)
        for (size_t s : lists[mth]) all.push_back({s, mth, w[mth]});
    if (all.empty()) return {};
    std::stable_sort(all.begin(), all.end(), [](const O& a, const O& b) { return a.sample < b.sample; });
    // Greedy clustering: join the FIRST cluster (creation order) holding ANY member within tol.
    std::vector<std::vector<const O*>> clusters;
    for (const O& o : all) {
        bool added = false;
        for (auto& cl : clusters) {
            for (const O* ex : cl) {
                const int64_t dd = (int64_t)(int32_t)o.sample - (int64_t)(int32_t)ex->sample;
                const uint64_t ad = (uint64_t)(dd < 0 ? -dd : dd);
                if ((size_t)ad <= tol) {
                    cl.push_back(&o);
                    added = true;
                    break;
                }
            }
            if (added) break;
        }
        if (!added) clusters.push_back({&o});
    }
    std::vector<OnsetCand> cands;
    float max_w = 0.0f;
    for (int i = 0; i < 4; i++) max_w += w[i];
    for (auto& cl : clusters) {
        size_t sum = 0;
        for (const O* o : cl) sum += o->sample;
        const size_t center = sum / cl.size();
        float tw = 0.0f;
        bool voted[4] = {false, false, false, false};
        for (const O* o : cl) {
            tw += o->weight;
            voted[o->method] = true;
        }
        uint32_t vb = 0;
        for (int i = 0; i < 4; i++) vb += voted[i];
        const float conf = max_w > 0.0f ? sd_clampf(tw / max_w, 0.0f, 1.0f) : 0.0f;
        cands.push_back({center, (float)center / (float)sr, conf, vb});
    }
    std::stable_sort(cands.begin(), cands.end(),
                     [](const OnsetCand& a, const OnsetCand& b) { return b.confidence < a.confidence; });
    return cands;
}

}  // namespace orc

namespace orc {

// hpss.rs:179-243: the median of every window [i - margin, i + margin] ∩ [0, n) along one row or
// column (sorted window; even length -> mean of the middle two times 0.5).  The sorted window is
// kept across positions (insert the entering value, erase the leaving one): the same multiset the
// reference collects and sorts per position, so the same median.
static void sliding_medians(const float* src, size_t n, size_t stride, size_t margin, float* dst, size_t dstride,
                            std::vector<float>& w) {
    w.clear();
    const size_t e0 = std::min(margin + 1, n);
    for (size_t k = 0; k < e0; k++) w.insert(std::upper_bound(w.begin(), w.end(), src[k * stride]), src[k * stride]);
    for (size_t i = 0; i < n; i++) {
        const size_t c = w.size(), mid = c / 2;
        dst[i * dstride] = c == 0 ? 0.0f : (c % 2 ? w[mid] : (w[mid - 1] + w[mid]) * 0.5f);
        if (i + margin + 1 < n) {
            const float v = src[(i + margin + 1) * stride];
            w.insert(std::upper_bound(w.begin(), w.end(), v), v);
        }
        if (i >= margin) w.erase(std::lower_bound(w.begin(), w.end(), src[(i - margin) * stride]));
    }
}

// src/features/onset/hpss.rs:71-172 (hpss_decompose, DEFAULT_ITERATIONS = 10)
void hpss_decompose(const Spec& m, size_t margin, Spec* H, Spec* P) {
    if (m.empty()) fail(SDSP_ERR_INVALID_INPUT, "Empty spectrogram");
    if (m.bins == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty frames");
    const size_t F = m.frames, B = m.bins;
    *H = m;
    *P = m;
    Spec hf = m, pf = m;
    std::vector<float> w;
    for (int it = 0; it < 10; it++) {
        const Spec hprev = *H, pprev = *P;
        for (size_t b = 0; b < B; b++)  // apply_horizontal_median_filter (:179-209)
            sliding_medians(H->d.data() + b, F, B, margin, hf.d.data() + b, B, w);
        for (size_t t = 0; t < F; t++)  // apply_vertical_median_filter (:213-243)
            sliding_medians(P->row(t), B, 1, margin, pf.row(t), 1, w);
        float max_change = 0.0f;
        for (size_t i = 0; i < F * B; i++) {
            const float orig = m.d[i], h = hf.d[i], p = pf.d[i];
            const float total = h + p;
            if (total > 1e-10f) {
                H->d[i] = orig * (h / total);
                P->d[i] = orig * (p / total);
            } else {
                H->d[i] = orig * 0.5f;
                P->d[i] = orig * 0.5f;
            }
            if (it > 0)
                max_change = sd_maxf(sd_maxf(max_change, sd_absf(H->d[i] - hprev.d[i])), sd_absf(P->d[i] - pprev.d[i]));
        }
        if (it > 0 && max_change < 1e-6f) break;
    }
}

// hpss.rs:290-372 (detect_hpss_onsets): energy flux of the percussive frames, percentile peaks
std::vector<size_t> hpss_onsets(const Spec& p, float pct) {
    if (p.empty()) return {};
    if (!(pct >= 0.0f && pct <= 1.0f)) fail(SDSP_ERR_INVALID_INPUT, "Threshold percentile must be in [0, 1]");
    if (p.frames < 2) return {};
    std::vector<float> e(p.frames);
    for (size_t t = 0; t < p.frames; t++) {
        float s = 0.0f;
        const float* r = p.row(t);
        for (size_t b = 0; b < p.bins; b++) s += r[b] * r[b];
        e[t] = s;
    }
    std::vector<float> flux(p.frames - 1);
    for (size_t i = 1; i < p.frames; i++) flux[i - 1] = sd_maxf(e[i] - e[i - 1], 0.0f);
    return peaks_over_percentile(flux, pct);
}

}  // namespace orc

// ctypes entry points for the HPSS unit tests (tests/test_oracle_hpss.py)
extern "C" int32_t sdsp_oracle_hpss(const float* spec, uint64_t frames, uint64_t bins, uint64_t margin, float* h,
                                    float* p) {
    orc::Spec s, H, P;
    s.frames = (size_t)frames;
    s.bins = (size_t)bins;
    s.d.assign(spec, spec + frames * bins);
    try {
        orc::hpss_decompose(s, (size_t)margin, &H, &P);
    } catch (const orc::AErr& e) {
        return e.code;
    }
    std::copy(H.d.begin(), H.d.end(), h);
    std::copy(P.d.begin(), P.d.end(), p);
    return 0;
}

extern "C" int64_t sdsp_oracle_hpss_onsets(const float* p, uint64_t frames, uint64_t bins, float pct, uint64_t* out,
                                           uint64_t cap) {
    orc::Spec s;
    s.frames = (size_t)frames;
    s.bins = (size_t)bins;
    s.d.assign(p, p + frames * bins);
    std::vector<size_t> on;
    try {
        on = orc::hpss_onsets(s, pct);
    } catch (const orc::AErr&) {
        return -1;
    }
    for (size_t i = 0; i < on.size() && i < cap; i++) out[i] = (uint64_t)on[i];
    return (int64_t)on.size();
}

// ---- unit probes (tests only; tests/test_oracle_units_onset.py) ----
namespace orc {
std::string g_probe_err;

void spec_from_rows(const float* d, size_t frames, size_t bins, const uint64_t* row_lens, Spec* out) {
    if (row_lens)
        for (size_t t = 0; t < frames; t++)
            if (row_lens[t] != row_lens[0])
                fail(SDSP_ERR_INVALID_INPUT, "Inconsistent frame lengths: frame 0 has " + std::to_string(row_lens[0]) +
                                                 " bins, frame " + std::to_string(t) + " has " +
                                                 std::to_string(row_lens[t]) + " bins");
    out->frames = frames;
    out->bins = frames ? bins : 0;
    out->d.assign(d, d + frames * bins);
}
}  // namespace orc

using namespace orc;

template <class V>
static int64_t put_list(const V& v, uint64_t* out, uint64_t cap) {
    for (size_t i = 0; i < v.size() && i < cap; i++) out[i] = (uint64_t)v[i];
    return (int64_t)v.size();
}

extern "C" {
const char* sdsp_oracle_probe_error(void) { return g_probe_err.c_str(); }

// detect_energy_flux_onsets (energy_flux.rs:67-243) -> onset sample positions
int64_t sdsp_oracle_energy_flux_onsets(const float* s, uint64_t n, uint64_t frame, uint64_t hop, float thr_db,
                                       uint64_t* out, uint64_t cap) {
    return probe_call([&]() -> int64_t { return put_list(energy_flux_onsets(s, n, frame, hop, thr_db), out, cap); });
}

// detect_spectral_flux_onsets (spectral_flux.rs:69-221) -> onset frame indices
int64_t sdsp_oracle_spectral_flux_onsets(const float* spec, uint64_t frames, uint64_t bins, const uint64_t* row_lens,
                                         float pct, uint64_t* out, uint64_t cap) {
    return probe_call([&]() -> int64_t {
        Spec m;
        spec_from_rows(spec, frames, bins, row_lens, &m);
        return put_list(spectral_flux_onsets(m, pct), out, cap);
    });
}

// detect_hfc_onsets (hfc.rs:76-214) -> onset frame indices
int64_t sdsp_oracle_hfc_onsets(const float* spec, uint64_t frames, uint64_t bins, const uint64_t* row_lens,
                               uint32_t sr, float pct, uint64_t* out, uint64_t cap) {
    return probe_call([&]() -> int64_t {
        Spec m;
        spec_from_rows(spec, frames, bins, row_lens, &m);
        return put_list(hfc_onsets(m, sr, pct), out, cap);
    });
}

// detect_and_trim (silence.rs:102-279): trim = [start, end) of the kept samples; regions =
// the silence map as (start, end) sample pairs; returns the region count
int64_t sdsp_oracle_detect_and_trim(const float* x, uint64_t n, uint32_t sr, float thr_db, uint32_t min_ms,
                                    uint64_t frame, uint64_t* trim, uint64_t* regions, uint64_t cap) {
    return probe_call([&]() -> int64_t {
        std::vector<float> v(x, x + n);
        std::vector<std::pair<size_t, size_t>> map;
        size_t ts = 0, te = 0;
        detect_and_trim(v, sr, thr_db, min_ms, (size_t)frame, &ts, &te, &map);
        trim[0] = ts;
        trim[1] = te;
        for (size_t i = 0; i < map.size() && i < cap; i++) {
            regions[2 * i] = map[i].first;
            regions[2 * i + 1] = map[i].second;
        }
        return (int64_t)map.size();
    });
}
}
