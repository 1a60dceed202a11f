// o_period.cpp — tempo estimation (TEST INFRASTRUCTURE, see oracle_internal.hpp).
//
// Follows src/features/period/{mod.rs, autocorrelation.rs, comb_filter.rs, candidate_filter.rs,
// novelty.rs, tempogram.rs, tempogram_fft.rs, tempogram_autocorr.rs, multi_resolution.rs}.
#include <algorithm>
#include <cmath>
#include <functional>

#include "oracle_internal.hpp"

namespace orc {

// Rust's stable sort for short slices is insertion sort (`insertion_sort_shift_left`); used
// where the reference's comparator is not a total order (candidate_filter.rs:392-440).
template <class T, class Less>
static void insertion_sort(std::vector<T>& v, Less is_less) {
    for (size_t i = 1; i < v.size(); i++) {
        T tmp = v[i];
        size_t j = i;
        while (j > 0 && is_less(tmp, v[j - 1])) {
            v[j] = v[j - 1];
            j--;
        }
        v[j] = tmp;
    }
}

static size_t next_pow2(size_t n) {
    size_t p = 1;
    while (p < n) p <<= 1;
    return p;
}

// =====================================================================================
// Legacy estimator (computed on every call, used only as the fallback; src/lib.rs:294-329)
// =====================================================================================

// autocorrelation.rs:229-268 (FFT size next_pow2(2n), |X|^2, inverse, /N, max(0))
static std::vector<float> acf_fft(const std::vector<float>& sig) {
    const size_t n = sig.size();
    const size_t N = next_pow2(2 * n);
    std::vector<Cx> x(N, Cx{0.0f, 0.0f});
    for (size_t i = 0; i < n; i++) x[i] = {sig[i], 0.0f};
    fft_complex(x);
    for (auto& c : x) c = {c.re * c.re - c.im * (-c.im), c.re * (-c.im) + c.im * c.re};  // x *= conj(x)
    // inverse: P is real (im == 0 exactly), so ifft(P) = conj(fft(conj(P))) has re = re(fft(P))
    for (auto& c : x) c.im = -c.im;
    fft_complex(x);
    const float scale = 1.0f / (float)N;
    std::vector<float> acf(n);
    for (size_t i = 0; i < n; i++) acf[i] = sd_maxf(x[i].re * scale, 0.0f);
    return acf;
}

// autocorrelation.rs:280-338
static std::vector<std::pair<size_t, float>> find_peaks_in_acf(const float* a, size_t len, size_t off) {
    std::vector<std::pair<size_t, float>> peaks;
    if (len == 0) return peaks;
    float mx = 0.0f;
    for (size_t i = 0; i < len; i++) mx = sd_maxf(mx, a[i]);
    if (mx < EPS) return peaks;
    const float min_prom = mx * 0.1f;
    const int64_t min_dist = 2;
    for (size_t i = 1; i + 1 < len; i++) {
        const float v = a[i];
        if (v > a[i - 1] && v > a[i + 1]) {
            const float prom = v - sd_maxf(a[i - 1], a[i + 1]);
            if (prom >= min_prom) {
                const size_t lag = i + off;
                const int64_t dl = (int64_t)(int32_t)lag - (int64_t)(int32_t)(peaks.empty() ? 0 : peaks.back().first);
                if (peaks.empty() || (dl < 0 ? -dl : dl) >= min_dist) {
                    peaks.push_back({lag, v});
                } else if (v > peaks.back().second) {
                    peaks.back() = {lag, v};
                }
            }
        }
    }
    std::stable_sort(peaks.begin(), peaks.end(), [](auto& x, auto& y) { return y.second < x.second; });
    return peaks;
}

// autocorrelation.rs:90-216
static std::vector<BpmCandidate> legacy_autocorr(const std::vector<size_t>& on, uint32_t sr, size_t hop,
                                                 float min_bpm, float max_bpm) {
    if (on.empty()) fail(SDSP_ERR_INVALID_INPUT, "Empty onset list");
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Invalid sample rate: 0");
    if (hop == 0) fail(SDSP_ERR_INVALID_INPUT, "Invalid hop size: 0");
    if (min_bpm <= 0.0f || max_bpm <= 0.0f || min_bpm >= max_bpm) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM range");
    if (on.size() < 2) return {};
    const size_t max_frame = *std::max_element(on.begin(), on.end()) / hop;
    const size_t L = max_frame + 1;
    if (L < 2) fail(SDSP_ERR_PROCESSING, "Signal too short for autocorrelation");
    std::vector<float> sig(L, 0.0f);
    for (size_t o : on)
        if (o / hop < L) sig[o / hop] = 1.0f;
    std::vector<float> acf = acf_fft(sig);
    const size_t lag_min = (size_t)sd_f2u64(std::ceil((60.0f * (float)sr) / (max_bpm * (float)hop)));
    const size_t lag_max = (size_t)sd_f2u64(std::floor((60.0f * (float)sr) / (min_bpm * (float)hop)));
    if (lag_min >= lag_max || lag_min >= acf.size() || lag_max >= acf.size()) return {};
    auto peaks = find_peaks_in_acf(acf.data() + lag_min, lag_max - lag_min + 1, lag_min);
    float max_acf = 0.0f;
    for (float v : acf) max_acf = sd_maxf(max_acf, v);
    std::vector<BpmCandidate> c;
    for (auto& pk : peaks) {
        const float bpm = (60.0f * (float)sr) / ((float)pk.first * (float)hop);
        if (bpm >= min_bpm && bpm <= max_bpm) {
            const float conf = max_acf > EPS ? sd_minf(pk.second / max_acf, 1.0f) : 0.0f;
            c.push_back({bpm, conf});
        }
    }
    std::stable_sort(c.begin(), c.end(), [](auto& a, auto& b) { return b.confidence < a.confidence; });
    return c;
}

// comb_filter.rs:342-397
static float comb_score(const std::vector<size_t>& on, uint32_t sr, float bpm, float tol) {
    if (on.empty()) return 0.0f;
    const float period = (60.0f * (float)sr) / bpm;
    if (period < 1.0f) fail(SDSP_ERR_NUMERICAL, "Invalid period");
    const float tol_s = period * tol;
    const float last = (float)on.back();
    const size_t nb = (size_t)sd_f2u64(std::ceil(last / period)) + 1;
    size_t aligned = 0;
    for (size_t bi = 0; bi < nb; bi++) {
        const float e = (float)bi * period;
        // min_by_key(|o| ((o as f32) - e).abs() as usize): FIRST minimum of the truncated key
        size_t best = 0;
        uint64_t bk = ~0ull;
        for (size_t k = 0; k < on.size(); k++) {
            const uint64_t key = sd_f2u64(sd_absf((float)on[k] - e));
            if (key < bk) {
                bk = key;
                best = k;
            }
        }
        const float dist = sd_absf((float)on[best] - e);
        if (dist <= tol_s) aligned++;
    }
    return nb > 0 ? (float)aligned / (float)nb : 0.0f;
}

// comb_filter.rs:90-240
static std::vector<BpmCandidate> legacy_comb(const std::vector<size_t>& on, uint32_t sr, float min_bpm,
                                             float max_bpm, float res) {
    if (on.empty()) fail(SDSP_ERR_INVALID_INPUT, "Empty onset list");
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Invalid sample rate: 0");
    if (min_bpm <= 0.0f || max_bpm <= 0.0f || min_bpm >= max_bpm) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM range");
    if (res <= 0.0f) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM resolution");
    if (on.size() < 2) return {};
    std::vector<size_t> s(on);
    std::sort(s.begin(), s.end());
    std::vector<std::pair<float, float>> c;
    float max_score = 0.0f;
    for (float bpm = min_bpm; bpm <= max_bpm + EPS; bpm += res) {
        const float at = sd_clampf(0.1f * (120.0f / bpm), 0.05f, 0.15f);
        const float sc = comb_score(s, sr, bpm, at);
        if (sc > max_score) max_score = sc;
        c.push_back({bpm, sc});
    }
    std::vector<BpmCandidate> r;
    for (auto& p : c) r.push_back({p.first, max_score > EPS ? p.second / max_score : 0.0f});
    std::stable_sort(r.begin(), r.end(), [](auto& a, auto& b) { return b.confidence < a.confidence; });
    std::vector<BpmCandidate> out;
    for (auto& x : r)
        if (x.confidence >= 0.1f) out.push_back(x);
    return out;
}

// candidate_filter.rs:40-97
static void boost_consensus(const std::vector<BpmCandidate>& a5, const std::vector<BpmCandidate>& c5,
                            std::vector<BpmEstimate>& est) {
    for (auto& e : est) {
        bool ad = false, cd = false, ah = false, ch = false;
        for (auto& a : a5) ad |= sd_absf(a.bpm - e.bpm) < 2.5f;
        for (auto& c : c5) cd |= sd_absf(c.bpm - e.bpm) < 2.5f;
        for (auto& a : a5) {
            const float r = sd_maxf(a.bpm / e.bpm, e.bpm / a.bpm);
            ah |= sd_absf(r - 2.0f) < 0.1f || sd_absf(r - 1.5f) < 0.1f || sd_absf(r - 0.75f) < 0.1f;
        }
        for (auto& c : c5) {
            const float r = sd_maxf(c.bpm / e.bpm, e.bpm / c.bpm);
            ch |= sd_absf(r - 2.0f) < 0.1f || sd_absf(r - 1.5f) < 0.1f || sd_absf(r - 0.75f) < 0.1f;
        }
        if (ad && cd)
            e.confidence *= 1.5f;
        else if ((ad && ch) || (cd && ah))
            e.confidence *= 1.3f;
        if (cd && e.bpm >= 60.0f && e.bpm <= 180.0f) e.confidence *= 1.4f;
    }
}

// candidate_filter.rs:147-442
static std::vector<BpmEstimate> merge_candidates(std::vector<BpmCandidate> ac, std::vector<BpmCandidate> comb,
                                                 float cents) {
    if (ac.empty() && comb.empty()) return {};
    const float tol_ratio = sd_exp2f(cents / 1200.0f);
    const size_t n3 = std::min<size_t>(3, comb.size());
    for (auto& a : ac) {
        for (size_t i = 0; i < n3; i++) {
            const auto& c = comb[i];
            const float ratio = a.bpm / c.bpm;
            const float rt = ratio / 2.0f;
            if (sd_absf(rt - 1.0f) < (tol_ratio - 1.0f)) {
                const bool corr = (c.bpm >= 60.0f && c.bpm <= 180.0f) || (a.bpm > 200.0f || a.bpm < 30.0f);
                if (corr) {
                    a.bpm = c.bpm;
                    break;
                }
            }
        }
    }
    for (auto& a : ac) {
        for (size_t i = 0; i < n3; i++) {
            const auto& c = comb[i];
            const float ratio = c.bpm / a.bpm;
            const float rt = ratio / 2.0f;
            if (sd_absf(rt - 1.0f) < (tol_ratio - 1.0f)) {
                if (c.bpm >= 60.0f && c.bpm <= 180.0f) {
                    a.bpm = c.bpm;
                    break;
                }
            }
        }
    }
    bool disagree = false;
    if (!ac.empty() && !comb.empty()) {
        const float d = sd_absf(ac[0].bpm - comb[0].bpm);
        disagree = d > 10.0f && d < 50.0f;
    }
    std::vector<BpmCandidate> al(ac.begin(), ac.begin() + std::min<size_t>(10, ac.size()));
    for (auto& c : ac) {
        if (c.bpm >= 60.0f && c.bpm <= 180.0f) {
            bool near = false;
            for (auto& x : al) near |= sd_absf(x.bpm - c.bpm) < 1.0f;
            if (!near) al.push_back(c);
        }
    }
    std::vector<BpmCandidate> cl(comb.begin(), comb.begin() + std::min<size_t>(10, comb.size()));
    struct G {
        float bpm, total;
        uint32_t count;
        float maxc;
    };
    std::vector<G> groups;
    auto add = [&](const BpmCandidate& c) {
        for (auto& g : groups) {
            if (sd_absf(c.bpm - g.bpm) <= 2.0f) {
                const uint32_t cnt = g.count;
                g.bpm = (g.bpm * (float)cnt + c.bpm) / (float)(cnt + 1);
                g.total += c.confidence;
                g.count += 1;
                g.maxc = sd_maxf(g.maxc, c.confidence);
                return;
            }
        }
        groups.push_back({c.bpm, c.confidence, 1, c.confidence});
    };
    for (auto& c : al) add(c);
    for (auto& c : cl) add(c);
    std::vector<BpmEstimate> est;
    for (auto& g : groups) {
        float conf;
        if (g.count >= 2) {
            const float avg = g.total / (float)g.count;
            conf = sd_minf((avg + g.maxc) / 2.0f * 1.2f, 1.0f);
        } else {
            conf = sd_minf(g.total, 1.0f);
        }
        if (disagree && g.count == 1) conf *= 0.7f;
        est.push_back({g.bpm, conf, g.count});
    }
    std::vector<BpmCandidate> a5(al.begin(), al.begin() + std::min<size_t>(5, al.size()));
    std::vector<BpmCandidate> c5(cl.begin(), cl.begin() + std::min<size_t>(5, cl.size()));
    boost_consensus(a5, c5, est);
    bool reasonable5 = false;
    for (size_t i = 0; i < std::min<size_t>(5, est.size()); i++)
        reasonable5 |= est[i].bpm >= 60.0f && est[i].bpm <= 180.0f;
    if (!reasonable5) {
        for (auto& e : est)
            if (e.bpm >= 60.0f && e.bpm <= 180.0f) {
                e.confidence *= 2.0f;
                break;
            }
    }
    auto cmp = [](const BpmEstimate& a, const BpmEstimate& b) -> int {
        const bool ai = a.bpm >= 60.0f && a.bpm <= 180.0f, bi = b.bpm >= 60.0f && b.bpm <= 180.0f;
        const float ae = ai ? a.confidence : a.confidence * 0.5f;
        const float be = bi ? b.confidence : b.confidence * 0.5f;
        int ec = (be < ae) ? -1 : (be > ae) ? 1 : 0;  // b_eff.partial_cmp(a_eff)
        if (sd_absf(ae - be) < 0.5f) {
            if (ai && !bi) return -1;
            if (!ai && bi) return 1;
        }
        if (ec != 0) return ec;
        return (b.method_agreement < a.method_agreement) ? -1 : (b.method_agreement > a.method_agreement) ? 1 : 0;
    };
    insertion_sort(est, [&](const BpmEstimate& a, const BpmEstimate& b) { return cmp(a, b) < 0; });
    return est;
}

// period/mod.rs:196-404 (estimate_bpm_internal)
bool estimate_bpm_legacy(const std::vector<size_t>& on, uint32_t sr, size_t hop, float min_bpm, float max_bpm,
                         float res, const Guardrails* g_in, BpmEstimate* out) {
    auto ac = legacy_autocorr(on, sr, hop, min_bpm, max_bpm);
    auto cb = legacy_comb(on, sr, min_bpm, max_bpm, res);
    Guardrails g{};
    if (g_in) {  // clamp_sane, mod.rs:88-121
        const Guardrails& s = *g_in;
        g.preferred_min = sd_minf(s.preferred_min, s.preferred_max);
        g.preferred_max = sd_maxf(s.preferred_min, s.preferred_max);
        g.soft_min = sd_minf(sd_minf(s.soft_min, s.soft_max), g.preferred_min);
        g.soft_max = sd_maxf(sd_maxf(s.soft_min, s.soft_max), g.preferred_max);
        g.mul_preferred = sd_isfinite_f(s.mul_preferred) ? sd_maxf(s.mul_preferred, 0.0f) : 0.0f;
        g.mul_soft = sd_isfinite_f(s.mul_soft) ? sd_maxf(s.mul_soft, 0.0f) : 0.0f;
        g.mul_extreme = sd_isfinite_f(s.mul_extreme) ? sd_maxf(s.mul_extreme, 0.0f) : 0.0f;
    }
    const float pmin = g_in ? g.preferred_min : 60.0f, pmax = g_in ? g.preferred_max : 180.0f;
    bool have_top = false;
    float top_pref = 0.0f;
    for (auto& c : ac)
        if (c.bpm >= pmin && c.bpm <= pmax) {
            have_top = true;
            top_pref = c.bpm;
            break;
        }
    std::vector<BpmEstimate> m = merge_candidates(ac, cb, 50.0f);
    if (g_in) {
        for (auto& e : m) {
            float mul;
            if (!sd_isfinite_f(e.bpm))
                mul = 0.0f;
            else if (e.bpm >= g.preferred_min && e.bpm <= g.preferred_max)
                mul = g.mul_preferred;
            else if (e.bpm >= g.soft_min && e.bpm <= g.soft_max)
                mul = g.mul_soft;
            else
                mul = g.mul_extreme;
            e.confidence *= mul;
        }
        std::stable_sort(m.begin(), m.end(), [](auto& a, auto& b) { return b.confidence < a.confidence; });
    }
    if (have_top) {
        for (size_t i = 0; i < m.size(); i++)
            if (sd_absf(m[i].bpm - top_pref) < 2.0f) {
                BpmEstimate e = m[i];
                m.erase(m.begin() + (long)i);
                m.insert(m.begin(), e);
                break;
            }
    }
    if (m.empty()) return false;
    *out = m[0];
    return true;
}

// =====================================================================================
// Novelty curves (novelty.rs)
// =====================================================================================

static void normalize_in_place(std::vector<float>& c) {  // novelty.rs:934-941
    float mx = 0.0f;
    for (float v : c) mx = sd_maxf(mx, v);
    if (mx > EPS)
        for (float& v : c) v /= mx;
}

// flux of a per-frame scalar (energy/HFC), positive differences, normalized (novelty.rs:512-530)
static std::vector<float> scalar_flux_norm(const std::vector<float>& e) {
    std::vector<float> f;
    for (size_t i = 1; i < e.size(); i++) f.push_back(sd_maxf(e[i] - e[i - 1], 0.0f));
    normalize_in_place(f);
    return f;
}

// superflux over the band [start,end) of log frames (novelty.rs:336-455; full band == [0,n))
static std::vector<float> superflux(const std::vector<float>& lf, size_t frames, size_t bins, size_t k,
                                    size_t start, size_t end) {
    std::vector<float> flux;
    if (frames < 2) return flux;
    k = std::max<size_t>(k, 1);
    for (size_t i = 1; i < frames; i++) {
        const float* prev = lf.data() + (i - 1) * bins;
        const float* curr = lf.data() + i * bins;
        float sum = 0.0f;
        for (size_t b = start; b < end; b++) {
            const size_t ls = std::max(b >= k ? b - k : 0, start);
            const size_t le = std::min(b + k + 1, end);
            float pm = 0.0f;
            for (size_t j = ls; j < le; j++) pm = sd_maxf(pm, prev[j]);
            const float d = sd_maxf(curr[b] - pm, 0.0f);
            sum += d * d;
        }
        flux.push_back(__builtin_sqrtf(sum));
    }
    normalize_in_place(flux);
    return flux;
}

static std::vector<float> local_mean_subtract(const std::vector<float>& x, size_t window) {  // :943-964
    if (x.empty() || window == 0) return x;
    const size_t half = std::max<size_t>(window, 1) / 2;
    std::vector<float> out(x.size());
    for (size_t i = 0; i < x.size(); i++) {
        const size_t s = i >= half ? i - half : 0, e = std::min(i + half + 1, x.size());
        float sum = 0.0f;
        for (size_t j = s; j < e; j++) sum += x[j];
        const float mean = sum / (float)(e - s);
        out[i] = sd_maxf(x[i] - mean, 0.0f);
    }
    return out;
}

static void smooth_ma(std::vector<float>& x, size_t window) {  // :966-983
    if (x.size() < 3 || window <= 1) return;
    const size_t half = std::max<size_t>(window, 1) / 2;
    std::vector<float> o(x);
    for (size_t i = 0; i < x.size(); i++) {
        const size_t s = i >= half ? i - half : 0, e = std::min(i + half + 1, x.size());
        float sum = 0.0f;
        for (size_t j = s; j < e; j++) sum += o[j];
        x[i] = sum / (float)(e - s);
    }
}

// novelty.rs:874-932
static std::vector<float> combine(const std::vector<float>& s, const std::vector<float>& e,
                                  const std::vector<float>& h, float ws_, float we_, float wh_, size_t lmw,
                                  size_t smw) {
    const size_t n = std::min(s.size(), std::min(e.size(), h.size()));
    if (n == 0) return {};
    const float ws = sd_maxf(ws_, 0.0f), we = sd_maxf(we_, 0.0f), wh = sd_maxf(wh_, 0.0f);
    const float wsum = sd_maxf(ws + we + wh, EPS);
    std::vector<float> c(n);
    for (size_t i = 0; i < n; i++) c[i] = (s[i] * ws + e[i] * we + h[i] * wh) / wsum;
    normalize_in_place(c);
    if (lmw > 1) c = local_mean_subtract(c, lmw);
    if (smw > 1) smooth_ma(c, smw);
    normalize_in_place(c);
    return c;
}

// Per-spectrogram state shared by the variants: ln(1+|X|) frames, energies, HFC
struct NovFrames {
    size_t frames, bins;
    std::vector<float> logf_;
};
static NovFrames log_frames(const Spec& m) {
    NovFrames nf{m.frames, m.bins, std::vector<float>(m.d.size())};
    for (size_t i = 0; i < m.d.size(); i++) nf.logf_[i] = sd_logf(1.0f + sd_maxf(m.d[i], 0.0f));
    return nf;
}
static std::vector<float> frame_energy(const Spec& m, size_t s, size_t e) {
    std::vector<float> r(m.frames);
    for (size_t t = 0; t < m.frames; t++) {
        const float* row = m.row(t);
        float acc = 0.0f;
        for (size_t b = s; b < e; b++) acc += row[b] * row[b];
        r[t] = acc;
    }
    return r;
}
static std::vector<float> frame_hfc(const Spec& m, size_t s, size_t e) {
    std::vector<float> r(m.frames);
    for (size_t t = 0; t < m.frames; t++) {
        const float* row = m.row(t);
        float acc = 0.0f;
        for (size_t b = s; b < e; b++) acc += (float)b * row[b] * row[b];
        r[t] = acc;
    }
    return r;
}

// MelFilterbank::new + apply_logmag + mel_superflux_novelty, novelty.rs:71-190, 553-609
static std::vector<float> mel_superflux(const Spec& m, const NovFrames& lf, uint32_t sr, size_t n_mels_in,
                                        float fmin_hz, float fmax_hz, size_t kk) {
    if (m.frames < 2) return {};
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate must be > 0");
    const size_t n_bins = m.bins;
    if (n_bins < 2) fail(SDSP_ERR_INVALID_INPUT, "Not enough FFT bins");
    const size_t n_mels = std::max<size_t>(n_mels_in, 4);
    const float nyq = (float)sr * 0.5f;
    const float fmin = sd_minf(sd_maxf(fmin_hz, 0.0f), sd_maxf(nyq, 1.0f));
    float fmax = fmax_hz;
    if (!(sd_isfinite_f(fmax) && fmax > 0.0f)) fmax = nyq;
    fmax = sd_clampf(fmax, fmin + 1.0f, nyq);
    const size_t fft_size = (n_bins - 1) * 2;
    const float fres = (float)sr / (float)fft_size;
    auto mel = [](float f) { return 2595.0f * sd_log10f(1.0f + (f / 700.0f)); };
    auto inv_mel = [](float v) { return 700.0f * (sd_powf(10.0f, v / 2595.0f) - 1.0f); };
    const float mmin = mel(fmin), mmax = mel(fmax);
    const float step = (mmax - mmin) / (float)(n_mels + 1);
    std::vector<size_t> bp(n_mels + 2);
    for (size_t i = 0; i < n_mels + 2; i++) {
        const float hz = inv_mel(mmin + step * (float)i);
        int64_t b = sd_f2i64(sd_roundf(hz / fres));
        b = std::max<int64_t>(0, std::min<int64_t>(b, (int64_t)n_bins - 1));
        bp[i] = (size_t)b;
    }
    for (size_t i = 1; i < bp.size(); i++)
        if (bp[i] <= bp[i - 1]) bp[i] = std::min(bp[i - 1] + 1, n_bins - 1);
    std::vector<std::vector<std::pair<size_t, float>>> contrib(n_bins);
    for (size_t mm = 0; mm < n_mels; mm++) {
        const size_t l = bp[mm], c = bp[mm + 1], r = bp[mm + 2];
        if (!(l < c && c < r)) continue;
        for (size_t b = l; b <= c; b++) {
            const float w = b == l ? 0.0f : ((float)b - (float)l) / ((float)c - (float)l);
            if (w > 0.0f) contrib[b].push_back({mm, w});
        }
        for (size_t b = c; b <= r; b++) {
            const float w = b == r ? 0.0f : ((float)r - (float)b) / ((float)r - (float)c);
            if (w > 0.0f) contrib[b].push_back({mm, w});
        }
    }
    std::vector<float> melf(m.frames * n_mels, 0.0f);
    for (size_t t = 0; t < m.frames; t++) {
        float* mv = melf.data() + t * n_mels;
        const float* lrow = lf.logf_.data() + t * n_bins;
        for (size_t b = 0; b < n_bins; b++) {
            const float v = lrow[b];  // (1.0 + x.max(0.0)).ln()
            if (v <= 0.0f) continue;
            for (auto& cw : contrib[b]) mv[cw.first] += v * cw.second;
        }
    }
    const size_t k = std::max<size_t>(kk, 1);
    std::vector<float> flux;
    for (size_t i = 1; i < m.frames; i++) {
        const float* prev = melf.data() + (i - 1) * n_mels;
        const float* curr = melf.data() + i * n_mels;
        float sum = 0.0f;
        for (size_t b = 0; b < n_mels; b++) {
            const size_t s = b >= k ? b - k : 0, e = std::min(b + k + 1, n_mels);
            float pm = 0.0f;
            for (size_t j = s; j < e; j++) pm = sd_maxf(pm, prev[j]);
            const float d = sd_maxf(curr[b] - pm, 0.0f);
            sum += d * d;
        }
        flux.push_back(__builtin_sqrtf(sum));
    }
    normalize_in_place(flux);
    return flux;
}

// =====================================================================================
// Tempograms (tempogram_fft.rs, tempogram_autocorr.rs)
// =====================================================================================
using Tg = std::vector<std::pair<float, float>>;  // (bpm, value), sorted by value desc

static Tg fft_tempogram(const std::vector<float>& nov, uint32_t sr, uint32_t hop, float min_bpm, float max_bpm) {
    if (nov.empty()) fail(SDSP_ERR_INVALID_INPUT, "Novelty curve is empty");
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate must be > 0");
    if (hop == 0) fail(SDSP_ERR_INVALID_INPUT, "Hop size must be > 0");
    if (min_bpm <= 0.0f || max_bpm <= min_bpm) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM range");
    const float frame_rate = (float)sr / (float)hop;
    float sum = 0.0f;
    for (float v : nov) sum += v;
    const float mean = sum / (float)nov.size();
    const size_t n = nov.size();
    const size_t P = next_pow2(n);
    std::vector<float> in(P, 0.0f);
    for (size_t i = 0; i < n; i++) {
        const float w = n > 1 ? sdsp_hann_f32((int)i, (int)n) : 1.0f;
        in[i] = (nov[i] - mean) * w;
    }
    Tg tg;
    const float fres = frame_rate / (float)P;
    if (P == 1) {  // size-1 FFT is the identity
        const float bpm = 0.0f * fres * 60.0f;
        if (bpm >= min_bpm && bpm <= max_bpm) tg.push_back({bpm, in[0] * in[0]});
        return tg;
    }
    std::vector<Cx> X;
    rfft(in.data(), P, X);
    for (size_t b = 0; b <= P / 2; b++) {
        const float bpm = (float)b * fres * 60.0f;
        if (bpm >= min_bpm && bpm <= max_bpm) tg.push_back({bpm, X[b].re * X[b].re + X[b].im * X[b].im});
    }
    std::stable_sort(tg.begin(), tg.end(), [](auto& a, auto& b) { return b.second < a.second; });
    return tg;
}

static Tg acf_tempogram(const std::vector<float>& nov, uint32_t sr, uint32_t hop, float min_bpm, float max_bpm,
                        float res) {
    if (nov.empty()) fail(SDSP_ERR_INVALID_INPUT, "Novelty curve is empty");
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate must be > 0");
    if (hop == 0) fail(SDSP_ERR_INVALID_INPUT, "Hop size must be > 0");
    if (min_bpm <= 0.0f || max_bpm <= min_bpm) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM range");
    if (res <= 0.0f) fail(SDSP_ERR_INVALID_INPUT, "BPM resolution must be > 0");
    const float frame_rate = (float)sr / (float)hop;
    Tg tg;
    const size_t n = nov.size();
    for (float bpm = min_bpm; bpm <= max_bpm; bpm += res) {
        const float bps = bpm / 60.0f;
        const float fpb = frame_rate / bps;
        const size_t lag = (size_t)sd_f2u64(fpb);
        float acc = 0.0f;
        int32_t cnt = 0;
        for (size_t i = 0; i + lag < n; i++) {
            acc += nov[i] * nov[i + lag];
            cnt++;
        }
        tg.push_back({bpm, cnt > 0 ? acc / (float)cnt : 0.0f});
    }
    std::stable_sort(tg.begin(), tg.end(), [](auto& a, auto& b) { return b.second < a.second; });
    return tg;
}

// find_best_bpm_fft / find_best_bpm_autocorr (tempogram_fft.rs:206-236, tempogram_autocorr.rs:192-222)
static bool find_best(const Tg& tg, float* bpm, float* conf) {
    if (tg.empty()) return false;
    *bpm = tg[0].first;
    const float best = tg[0].second;
    if (tg.size() > 1) {
        *conf = best > EPS ? sd_clampf(sd_maxf(best - tg[1].second, 0.0f) / best, 0.0f, 1.0f) : 0.0f;
    } else {
        *conf = 0.5f;
    }
    return true;
}

static float lookup_nearest(const Tg& tg, float bpm, float tol) {  // tempogram.rs:521-532
    float bd = SD_INF_F, bv = 0.0f;
    for (auto& e : tg) {
        const float d = sd_absf(e.first - bpm);
        if (d <= tol && d < bd) {
            bd = d;
            bv = e.second;
        }
    }
    return bv;
}

std::vector<float> combined_full_novelty(const Spec& m, uint32_t sr, const BandCfg& c) {
    (void)sr;
    NovFrames lf = log_frames(m);
    auto sf = superflux(lf.logf_, m.frames, m.bins, c.superflux_k, 0, m.bins);
    auto en = scalar_flux_norm(frame_energy(m, 0, m.bins));
    auto hf = scalar_flux_norm(frame_hfc(m, 0, m.bins));
    return combine(sf, en, hf, c.nw_spectral, c.nw_energy, c.nw_hfc, c.local_mean_window, c.smooth_window);
}

// tempogram.rs:255-775 (estimate_bpm_tempogram_impl); cands = full scored list (callers truncate)
void tempogram_impl(const Spec& m, uint32_t sr, uint32_t hop, float min_bpm, float max_bpm, float res,
                    const BandCfg* band, BpmEstimate* est, std::vector<TempoCand>* cands_out) {
    const size_t n_bins = m.frames ? m.bins : 0;
    if (n_bins == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty magnitude frames");
    const size_t fft_size = std::max<size_t>((n_bins >= 1 ? n_bins - 1 : 0) * 2, 2);
    const float fres = (float)sr / (float)fft_size;
    auto hz_to_bin = [&](float f) -> size_t {
        if (!sd_isfinite_f(f) || f <= 0.0f || !sd_isfinite_f(fres) || fres <= 0.0f) return 0;
        int64_t b = sd_f2i64(sd_roundf(f / fres));
        return (size_t)std::max<int64_t>(0, std::min<int64_t>(b, (int64_t)n_bins - 1));
    };
    struct Variant {
        const char* name;
        float w;
        Tg fft, ac;
        float max_fft, max_ac;
    };
    const size_t sf_k = band ? band->superflux_k : 4;
    NovFrames lf = log_frames(m);
    std::vector<float> nov_full;
    {
        auto sf = superflux(lf.logf_, m.frames, m.bins, sf_k, 0, m.bins);
        auto en = m.frames >= 2 ? scalar_flux_norm(frame_energy(m, 0, m.bins)) : std::vector<float>{};
        auto hf = m.frames >= 2 ? scalar_flux_norm(frame_hfc(m, 0, m.bins)) : std::vector<float>{};
        if (band)
            nov_full = combine(sf, en, hf, band->nw_spectral, band->nw_energy, band->nw_hfc, band->local_mean_window,
                               band->smooth_window);
        else
            nov_full = combine(sf, en, hf, 0.5f, 0.3f, 0.2f, 16, 5);
    }
    if (nov_full.empty()) fail(SDSP_ERR_PROCESSING, "Novelty curve is empty after extraction");
    auto mk = [&](const char* name, float w, const std::vector<float>& nov) {
        Variant v{name, w, fft_tempogram(nov, sr, hop, min_bpm, max_bpm), acf_tempogram(nov, sr, hop, min_bpm, max_bpm, res),
                  0.0f, 0.0f};
        v.max_fft = sd_maxf(v.fft.empty() ? 1.0f : v.fft[0].second, 1e-12f);
        v.max_ac = sd_maxf(v.ac.empty() ? 1.0f : v.ac[0].second, 1e-12f);
        return v;
    };
    std::vector<Variant> seeds;
    seeds.push_back(mk("full", band ? band->w_full : 1.0f, nov_full));
    float fft_pb = 0.0f, fft_pc = 0.0f, ac_pb = 0.0f, ac_pc = 0.0f;
    if (!find_best(seeds[0].fft, &fft_pb, &fft_pc)) fft_pb = 0.0f, fft_pc = 0.0f;
    if (!find_best(seeds[0].ac, &ac_pb, &ac_pc)) ac_pb = 0.0f, ac_pc = 0.0f;
    if (band && band->enabled) {
        const size_t b0 = std::min<size_t>(1, n_bins >= 1 ? n_bins - 1 : 0);
        const size_t bl = std::max(hz_to_bin(band->low_max_hz), b0);
        const size_t bm = std::max(hz_to_bin(band->mid_max_hz), bl + 1);
        size_t bh = band->high_max_hz > 0.0f ? std::max(hz_to_bin(band->high_max_hz), bm + 1) : n_bins;
        bh = std::min(bh, n_bins);
        struct B {
            const char* n;
            size_t s, e;
            float w;
        } bands[3] = {{"low", b0, bl, band->w_low}, {"mid", bl, bm, band->w_mid}, {"high", bm, bh, band->w_high}};
        for (auto& b : bands) {
            if (!(sd_isfinite_f(b.w) && b.w > 0.0f)) continue;
            if (b.e <= b.s + 1) continue;
            const size_t s = std::min(b.s, n_bins), e = std::min(b.e, n_bins);
            std::vector<float> sp, en, hf;
            if (m.frames >= 2 && e > s + 1) {
                sp = superflux(lf.logf_, m.frames, m.bins, sf_k, s, e);
                en = scalar_flux_norm(frame_energy(m, s, e));
                hf = scalar_flux_norm(frame_hfc(m, s, e));
            }
            auto nov = combine(sp, en, hf, band->nw_spectral, band->nw_energy, band->nw_hfc, band->local_mean_window,
                               band->smooth_window);
            if (nov.empty()) continue;
            seeds.push_back(mk(b.n, b.w, nov));
        }
    }
    if (band && band->enable_mel) {
        auto mc = mel_superflux(m, lf, sr, band->mel_n_mels, band->mel_fmin_hz, band->mel_fmax_hz,
                                band->mel_max_filter_bins);
        if (!mc.empty()) seeds.push_back(mk("mel", band->w_mel, mc));
    }
    const bool seed_only = band ? band->seed_only : true;
    std::vector<const Variant*> score_v;
    for (auto& v : seeds)
        if (!seed_only || std::strcmp(v.name, "full") == 0) score_v.push_back(&v);
    const float support_thr = sd_clampf(band ? band->support_threshold : 0.25f, 0.0f, 1.0f);
    const float bonus = sd_maxf(band ? band->consensus_bonus : 0.0f, 0.0f);
    float w_sum = 0.0f;
    for (auto* v : score_v) w_sum += sd_maxf(v->w, 0.0f);
    w_sum = sd_maxf(w_sum, 1e-6f);
    bool all_empty = true;
    for (auto& v : seeds) all_empty &= v.fft.empty() && v.ac.empty();
    if (all_empty) fail(SDSP_ERR_PROCESSING, "Both FFT and autocorrelation tempograms are empty");

    std::vector<float> seed_bpms;
    for (auto& v : seeds) {
        for (size_t i = 0; i < std::min<size_t>(8, v.fft.size()); i++) seed_bpms.push_back(v.fft[i].first);
        for (size_t i = 0; i < std::min<size_t>(8, v.ac.size()); i++) seed_bpms.push_back(v.ac[i].first);
    }
    if (fft_pb > 0.0f) seed_bpms.push_back(fft_pb);
    if (ac_pb > 0.0f) seed_bpms.push_back(ac_pb);
    const float FACT[7] = {1.0f, 0.5f, 2.0f, 1.0f / 3.0f, 3.0f, 2.0f / 3.0f, 3.0f / 2.0f};
    std::vector<float> c;
    for (float b : seed_bpms)
        for (float f : FACT) {
            const float x = b * f;
            if (sd_isfinite_f(x) && x >= min_bpm && x <= max_bpm) c.push_back(x);
        }
    std::stable_sort(c.begin(), c.end(), [](float a, float b) { return a < b; });
    std::vector<float> uniq;
    for (float b : c) {
        if (!uniq.empty() && sd_absf(b - uniq.back()) < 0.75f) continue;
        uniq.push_back(b);
    }
    const float ac_tol = sd_maxf(res, 0.5f);
    const bool bonus_on = bonus > 0.0f && band && (band->enabled || band->enable_mel);
    std::vector<TempoCand> scored;
    for (float bpm : uniq) {
        float fa = 0.0f, aa = 0.0f;
        for (auto* v : score_v) {
            if (v->w <= 0.0f) continue;
            const float fv = lookup_nearest(v->fft, bpm, 0.75f);
            const float av = lookup_nearest(v->ac, bpm, ac_tol);
            fa += v->w * sd_clampf(fv / v->max_fft, 0.0f, 1.0f);
            aa += v->w * sd_clampf(av / v->max_ac, 0.0f, 1.0f);
        }
        const float fn = sd_clampf(fa / w_sum, 0.0f, 1.0f);
        const float an = sd_clampf(aa / w_sum, 0.0f, 1.0f);
        float score = 0.55f * an + 0.45f * fn;
        if (bonus_on) {
            uint32_t sb = 0;
            for (auto& v : seeds) {
                if (std::strcmp(v.name, "full") == 0) continue;
                const float sff = sd_clampf(lookup_nearest(v.fft, bpm, 0.75f) / v.max_fft, 0.0f, 1.0f);
                const float sac = sd_clampf(lookup_nearest(v.ac, bpm, ac_tol) / v.max_ac, 0.0f, 1.0f);
                if (sd_maxf(sff, sac) >= support_thr) sb++;
            }
            if (sb >= 2) score *= 1.0f + bonus * ((float)sb - 1.0f);
        }
        if (bpm > 180.0f)
            score *= 0.80f;
        else if (bpm < 60.0f)
            score *= 0.90f;
        scored.push_back({bpm, score, fn, an, false});
    }
    std::stable_sort(scored.begin(), scored.end(), [](auto& a, auto& b) { return b.score < a.score; });
    if (scored.empty()) fail(SDSP_ERR_PROCESSING, "No BPM candidates could be scored");
    TempoCand best = scored[0];
    if (best.bpm > 180.0f) {
        const float folded = best.bpm / 2.0f;
        if (folded >= min_bpm && folded <= max_bpm) {
            for (auto& fc : scored) {
                if (sd_absf(fc.bpm - folded) < 0.75f) {
                    const float eps = 1e-6f;
                    const float ar = (best.autocorr_norm + eps) / (fc.autocorr_norm + eps);
                    const float fr = (best.fft_norm + eps) / (fc.fft_norm + eps);
                    if (!(ar > 2.0f && fr > 2.0f)) best = fc;
                    break;
                }
            }
        }
    }
    float conf = 0.0f;
    if (best.score > 1e-12f) {
        const float ss = scored.size() > 1 ? scored[1].score : 0.0f;
        conf = sd_clampf(sd_maxf(best.score - ss, 0.0f) / best.score, 0.0f, 1.0f);
    }
    uint32_t agree = 0;
    if (fft_pb > 0.0f && sd_absf(fft_pb - best.bpm) < 2.0f) agree++;
    if (ac_pb > 0.0f && sd_absf(ac_pb - best.bpm) < 2.0f) agree++;
    *est = {best.bpm, conf, agree};
    if (cands_out) {
        for (auto& s : scored) s.selected = sd_absf(s.bpm - best.bpm) < 0.75f;
        *cands_out = scored;
    }
}

// =====================================================================================
// Multi-resolution escalation, multi_resolution.rs:205-901
// =====================================================================================

static float lookup_c(const std::vector<TempoCand>& c, float bpm, float tol) {  // :285-296
    float bd = SD_INF_F, bs = 0.0f;
    for (auto& x : c) {
        const float d = sd_absf(x.bpm - bpm);
        if (d <= tol && d < bd) {
            bd = d;
            bs = x.score;
        }
    }
    return bs;
}

static float beat_contrast(const std::vector<float>& nov, uint32_t sr, uint32_t hop, float bpm) {  // :580-678
    if (nov.size() < 16 || !(sd_isfinite_f(bpm) && bpm > 0.0f) || sr == 0 || hop == 0) return 0.0f;
    const float fpb = (60.0f * (float)sr) / (bpm * (float)hop);
    if (!sd_isfinite_f(fpb) || fpb < 3.0f) return 0.0f;
    const int64_t period_i = sd_f2i64(sd_roundf(fpb));
    if (!(period_i >= 3 && period_i <= 512)) return 0.0f;
    const size_t period = (size_t)period_i, w = 2, n = nov.size();
    float total = 0.0f;
    for (float v : nov) total += v;
    total = sd_maxf(total, 1e-6f);
    auto wmax = [&](size_t i) {
        const size_t s = i >= w ? i - w : 0, e = std::min(i + w + 1, n);
        float mx = 0.0f;
        for (size_t j = s; j < e; j++) mx = sd_maxf(mx, nov[j]);
        return mx;
    };
    float best = -1e9f;
    for (size_t ph = 0; ph < period; ph++) {
        float bs = 0.0f, hs = 0.0f, ts = 0.0f;
        uint32_t bn = 0, hn = 0, tn = 0;
        for (size_t i = ph; i < n; i += period) {
            bs += wmax(i);
            bn++;
            if (period >= 6) {
                const size_t j = i + period / 2;
                if (j < n) {
                    hs += wmax(j);
                    hn++;
                }
            }
            if (period >= 9) {
                for (size_t fr = 1; fr <= 2; fr++) {
                    const size_t j = i + (period * fr) / 3;
                    if (j < n) {
                        ts += wmax(j);
                        tn++;
                    }
                }
            }
        }
        const float bm = bn > 0 ? bs / (float)bn : 0.0f;
        const float hm = hn > 0 ? hs / (float)hn : 0.0f;
        const float tm = tn > 0 ? ts / (float)tn : 0.0f;
        const float contrast = bm - 0.60f * hm - 0.40f * tm;
        const float score = sd_clampf(contrast / sd_maxf(total / (float)n, 1e-6f), -10.0f, 10.0f);
        best = sd_maxf(best, score);
    }
    return best;
}

static void total_support(const std::vector<TempoCand>& c256, const std::vector<TempoCand>& c512,
                          const std::vector<TempoCand>& c1024, float bpm, float tol, float* s, uint32_t* a) {
    const float s256 = lookup_c(c256, bpm, tol), s512 = lookup_c(c512, bpm, tol), s1024 = lookup_c(c1024, bpm, tol);
    *a = (s256 > 0.0f) + (s512 > 0.0f) + (s1024 > 0.0f);
    *s = s256 + s512 + s1024;
}

void multi_resolution(const std::vector<float>& samples, uint32_t sr, size_t frame_size, float min_bpm,
                      float max_bpm, float res, size_t top_k_in, float w512, float w256, float w1024,
                      float structural_discount, float dt, float margin_thr, bool human_prior, const BandCfg* band,
                      BpmEstimate* est, std::vector<TempoCand>* c512_out) {
    (void)structural_discount;  // only used by the debug dump (:316-318)
    if (samples.size() < frame_size) fail(SDSP_ERR_INVALID_INPUT, "Audio too short for STFT");
    const size_t top_k = std::max<size_t>(top_k_in, 1);
    const size_t aux_k = std::min<size_t>(std::max<size_t>(top_k * 4, 25), 200);
    const float tol = sd_maxf(2.0f, res);
    Spec h256 = compute_stft(samples.data(), samples.size(), frame_size, 256);
    Spec h512 = compute_stft(samples.data(), samples.size(), frame_size, 512);
    Spec h1024 = compute_stft(samples.data(), samples.size(), frame_size, 1024);
    const BandCfg* cfg = (band && (band->enabled || band->enable_mel || band->consensus_bonus > 0.0f)) ? band : nullptr;
    auto call = [&](const Spec& s, uint32_t hop, size_t k, std::vector<TempoCand>* out) {
        BpmEstimate e;
        tempogram_impl(s, sr, hop, min_bpm, max_bpm, res, cfg, &e, out);
        if (k == 0)
            out->clear();
        else if (out->size() > k)
            out->resize(k);
    };
    std::vector<TempoCand> c256, c512, c1024;
    call(h256, 256, aux_k, &c256);
    call(h512, 512, top_k, &c512);
    call(h1024, 1024, aux_k, &c1024);
    struct Hyp {
        float bpm, score;
    };
    std::vector<Hyp> hyps;
    for (size_t ti = 0; ti < std::min(top_k, c512.size()); ti++) {
        const float t = c512[ti].bpm;
        if (!(sd_isfinite_f(t) && t > 0.0f)) continue;
        const float st512 = lookup_c(c512, t, tol), st256 = lookup_c(c256, t, tol), st1024 = lookup_c(c1024, t, tol);
        const float s2512 = lookup_c(c512, t * 2.0f, tol), s2256 = lookup_c(c256, t * 2.0f, tol),
                    s21024 = lookup_c(c1024, t * 2.0f, tol);
        const float sh512 = lookup_c(c512, t * 0.5f, tol), sh256 = lookup_c(c256, t * 0.5f, tol),
                    sh1024 = lookup_c(c1024, t * 0.5f, tol);
        const float h_t = w512 * st512 + w256 * st256 + w1024 * st1024;
        float h_2t = w512 * (dt * st512 + (1.0f - dt) * s2512) + w256 * s2256 + w1024 * s21024;
        float h_h = w512 * (dt * st512 + (1.0f - dt) * sh512) + w256 * sh256 + w1024 * sh1024;
        if (st1024 > sh1024 * 1.02f) h_h *= 0.90f;
        if (st1024 > s21024 * 1.02f) h_2t *= 0.90f;
        const float eps = 1e-6f;
        const float r2 = (s2256 + eps) / (st256 + eps);
        if (r2 < 1.10f) h_2t *= 0.75f;
        if (r2 < 1.00f) h_2t *= 0.75f;
        const float rh = (sh1024 + eps) / (st1024 + eps);
        if (rh < 1.10f) h_h *= 0.75f;
        if (rh < 1.00f) h_h *= 0.75f;
        std::vector<Hyp> local;
        for (Hyp h : {Hyp{t, h_t}, Hyp{t * 2.0f, h_2t}, Hyp{t * 0.5f, h_h}})
            if (h.bpm >= min_bpm && h.bpm <= max_bpm) local.push_back(h);
        for (auto& h : local) {
            if (h.bpm > 210.0f)
                h.score *= 0.80f;
            else if (h.bpm > 180.0f)
                h.score *= 0.90f;
            else if (h.bpm < 60.0f)
                h.score *= 0.92f;
        }
        std::stable_sort(local.begin(), local.end(), [](auto& a, auto& b) { return b.score < a.score; });
        if (local.empty()) continue;
        const float bb = local[0].bpm, bsc = local[0].score;
        const float ss = local.size() > 1 ? local[1].score : 0.0f;
        const float margin = bsc - ss;
        float cb = bb, cs = bsc;
        if (sd_absf(cb - t) > 1e-3f && margin < margin_thr) {
            cb = t;
            cs = h_t;
        }
        if (margin < margin_thr && human_prior && cb >= 70.0f && cb <= 180.0f && margin < 0.05f) cs += 0.05f;
        hyps.push_back({cb, cs});
    }
    if (hyps.empty()) fail(SDSP_ERR_PROCESSING, "Multi-resolution fusion produced no hypotheses");
    std::stable_sort(hyps.begin(), hyps.end(), [](auto& a, auto& b) { return b.score < a.score; });
    std::vector<Hyp> uniq;
    for (auto& h : hyps) {
        bool dup = false;
        for (auto& u : uniq) dup |= sd_absf(u.bpm - h.bpm) < 0.75f;
        if (dup) continue;
        uniq.push_back(h);
        if (uniq.size() >= 8) break;
    }
    Hyp best = uniq[0];
    std::vector<float> nov512;
    if (band) nov512 = combined_full_novelty(h512, sr, *band);
    if (best.bpm >= 170.0f) {  // fold-down :698-724
        const float half = best.bpm * 0.5f;
        if (half >= 70.0f && half <= 120.0f) {
            float sb, sh;
            uint32_t ab, ah;
            total_support(c256, c512, c1024, best.bpm, tol, &sb, &ab);
            total_support(c256, c512, c1024, half, tol, &sh, &ah);
            const float ratio = sb > 0.0f ? sh / sb : 0.0f;
            if (ah >= 3 && sh > 0.0f && sb > 0.0f && ratio >= 0.45f) best = {half, sh};
        }
    }
    if (best.bpm <= 80.0f) {  // fold-up :727-751
        const float dbl = best.bpm * 2.0f;
        if (dbl >= 70.0f && dbl <= 180.0f) {
            float sb, sd;
            uint32_t ab, ad;
            total_support(c256, c512, c1024, best.bpm, tol, &sb, &ab);
            total_support(c256, c512, c1024, dbl, tol, &sd, &ad);
            const float ratio = sb > 0.0f ? sd / sb : 0.0f;
            if (ad >= 2 && sd > 0.0f && sb > 0.0f && ratio >= 0.55f) best = {dbl, sd};
        }
    }
    if (band && best.bpm >= 70.0f && best.bpm <= 180.0f && !nov512.empty()) {  // triplet family :764-867
        const float fam_f[5] = {1.0f, 3.0f / 2.0f, 2.0f / 3.0f, 4.0f / 3.0f, 3.0f / 4.0f};
        struct Fam {
            float bpm, support, align;
        };
        std::vector<Fam> fams;
        for (float f : fam_f) {
            const float bpm = best.bpm * f;
            if (!(sd_isfinite_f(bpm) && bpm >= min_bpm && bpm <= max_bpm)) continue;
            if (!(bpm >= 70.0f && bpm <= 180.0f)) continue;
            float sup;
            uint32_t ag;
            total_support(c256, c512, c1024, bpm, tol, &sup, &ag);
            if (ag < 2 || sup <= 0.0f) continue;
            fams.push_back({bpm, sup, beat_contrast(nov512, sr, 512, bpm)});
        }
        if (fams.size() >= 2) {
            float bs = 0.0f;
            for (auto& f : fams) bs = sd_maxf(bs, f.support);
            bs = sd_maxf(bs, 1e-6f);
            float max_alt = 0.0f;
            for (auto& f : fams)
                if (sd_absf(f.bpm - best.bpm) > 0.75f) max_alt = sd_maxf(max_alt, f.support / bs);
            if (max_alt >= 0.45f) {
                Fam chosen = fams[0];
                float cscore = -1e9f;
                for (auto& f : fams) {
                    const float sn = sd_clampf(f.support / bs, 0.0f, 1.0f);
                    const float sc = f.align + 0.35f * sn;
                    if (sc > cscore) {
                        chosen = f;
                        cscore = sc;
                    }
                }
                const float cur_align = beat_contrast(nov512, sr, 512, best.bpm);
                if (sd_absf(chosen.bpm - best.bpm) > 0.75f && chosen.align >= cur_align + 0.40f)
                    best = {chosen.bpm, chosen.support};
            }
        }
    }
    const float second = uniq.size() > 1 ? uniq[1].score : 0.0f;
    const float conf =
        best.score > 1e-6f ? sd_clampf(sd_maxf(best.score - second, 0.0f) / best.score, 0.0f, 1.0f) : 0.0f;
    uint32_t agree = (lookup_c(c256, best.bpm, tol) > 0.0f) + (lookup_c(c512, best.bpm, tol) > 0.0f) +
                     (lookup_c(c1024, best.bpm, tol) > 0.0f);
    for (auto& c : c512) c.selected = sd_absf(c.bpm - best.bpm) < 0.75f;
    *est = {best.bpm, conf, agree};
    if (c512_out) *c512_out = c512;
}

}  // namespace orc

// find_best_bpm_fft / find_best_bpm_autocorr probe (tests only): tempogram already sorted by
// value descending, as both tempogram builders return it.  Returns 0 for an empty tempogram.
extern "C" int32_t sdsp_oracle_find_best(const float* bpm, const float* val, int32_t n, float* out_bpm,
                                         float* out_val, float* out_conf) {
    orc::Tg tg;
    for (int32_t i = 0; i < n; i++) tg.push_back({bpm[i], val[i]});
    float b = 0.0f, c = 0.0f;
    if (!orc::find_best(tg, &b, &c)) return 0;
    *out_bpm = b;
    *out_val = tg[0].second;
    *out_conf = c;
    return 1;
}


// ctypes entry point for the legacy-estimator unit tests (tests/test_oracle_legacy.py).
// which: 0 autocorrelation candidates (autocorrelation.rs:90-216), 1 comb-filter candidates
// (comb_filter.rs:96-215), 2 the estimate (mod.rs:196-404; g7 = guardrails or null), 3
// merge_bpm_candidates (candidate_filter.rs:147-442) of in[0..n_ac) and in[n_ac..n_ac+n_comb).
// Returns the number of entries written, or -(AnalysisError code).
extern "C" int64_t sdsp_oracle_legacy(int32_t which, const uint64_t* on, uint64_t n, uint32_t sr, uint64_t hop,
                                      float min_bpm, float max_bpm, float res, const float* in_bpm,
                                      const float* in_conf, uint64_t n_ac, uint64_t n_comb, const float* g7,
                                      float* out_bpm, float* out_conf, uint32_t* out_agree, uint64_t cap) {
    using namespace orc;
    std::vector<size_t> o(on, on + n);
    std::vector<BpmEstimate> est;
    try {
        if (which == 0 || which == 1) {
            auto c = which == 0 ? legacy_autocorr(o, sr, (size_t)hop, min_bpm, max_bpm)
                                : legacy_comb(o, sr, min_bpm, max_bpm, res);
            for (auto& x : c) est.push_back({x.bpm, x.confidence, 0});
        } else if (which == 2) {
            BpmEstimate e{};
            Guardrails g{};
            if (g7) g = {g7[0], g7[1], g7[2], g7[3], g7[4], g7[5], g7[6]};
            if (estimate_bpm_legacy(o, sr, (size_t)hop, min_bpm, max_bpm, res, g7 ? &g : nullptr, &e)) est.push_back(e);
        } else {
            std::vector<BpmCandidate> a, c;
            for (uint64_t i = 0; i < n_ac; i++) a.push_back({in_bpm[i], in_conf[i]});
            for (uint64_t i = 0; i < n_comb; i++) c.push_back({in_bpm[n_ac + i], in_conf[n_ac + i]});
            est = merge_candidates(a, c, 50.0f);
        }
    } catch (const AErr& e) {
        return -(int64_t)e.code;
    }
    for (size_t i = 0; i < est.size() && i < cap; i++) {
        out_bpm[i] = est[i].bpm;
        out_conf[i] = est[i].confidence;
        out_agree[i] = est[i].method_agreement;
    }
    return (int64_t)est.size();
}

// =====================================================================================
// Unit probes (tests only; tests/test_oracle_units_tempo.py): the reference functions at the
// granularity of its own unit tests, built from the restatement above.
// =====================================================================================
namespace orc {

static void check_bins(const Spec& m) {  // validate_spectrogram (novelty.rs:39-60); raggedness: spec_from_rows
    if (m.frames >= 2 && m.bins == 0) fail(SDSP_ERR_INVALID_INPUT, "Empty magnitude frames");
}

std::vector<float> superflux_novelty(const Spec& m, size_t k) {
    if (m.frames < 2) return {};
    check_bins(m);
    if (m.bins == 0) return {};
    NovFrames lf = log_frames(m);
    return superflux(lf.logf_, m.frames, m.bins, k, 0, m.bins);
}

std::vector<float> energy_flux_novelty(const Spec& m) {
    if (m.frames < 2) return {};
    check_bins(m);
    return scalar_flux_norm(frame_energy(m, 0, m.bins));
}

std::vector<float> hfc_novelty(const Spec& m, uint32_t sr) {
    if (m.frames == 0) return {};
    if (sr == 0) fail(SDSP_ERR_INVALID_INPUT, "Sample rate must be > 0");
    if (m.frames < 2) return {};
    check_bins(m);
    return scalar_flux_norm(frame_hfc(m, 0, m.bins));
}

// per-frame max-normalised half-wave L2 flux, normalised by its max (novelty.rs:222-334)
std::vector<float> spectral_flux_novelty(const Spec& m) {
    if (m.frames < 2) return {};
    check_bins(m);
    const size_t B = m.bins;
    std::vector<float> norm(m.d.size(), 0.0f);
    for (size_t t = 0; t < m.frames; t++) {
        const float* r = m.row(t);
        float mx = 0.0f;
        for (size_t b = 0; b < B; b++) mx = sd_maxf(mx, r[b]);
        if (mx > EPS)
            for (size_t b = 0; b < B; b++) norm[t * B + b] = r[b] / mx;
    }
    std::vector<float> flux;
    for (size_t t = 1; t < m.frames; t++) {
        float sum = 0.0f;
        for (size_t b = 0; b < B; b++) {
            const float d = sd_maxf(norm[t * B + b] - norm[(t - 1) * B + b], 0.0f);
            sum += d * d;
        }
        flux.push_back(__builtin_sqrtf(sum));
    }
    normalize_in_place(flux);
    return flux;
}

std::vector<float> combined_novelty_params(const std::vector<float>& s, const std::vector<float>& e,
                                           const std::vector<float>& h, float ws, float we, float wh, size_t lmw,
                                           size_t smw) {
    return combine(s, e, h, ws, we, wh, lmw, smw);
}

}  // namespace orc

using namespace orc;

extern "C" {

static int64_t put_curve(const std::vector<float>& v, float* out) {
    if (out) std::memcpy(out, v.data(), v.size() * sizeof(float));
    return (int64_t)v.size();
}

// kind 0 spectral_flux_novelty, 1 energy_flux_novelty, 2 hfc_novelty, 3 superflux_novelty(k);
// out holds frames - 1 values; returns the curve length
int64_t sdsp_oracle_novelty(int32_t kind, const float* spec, uint64_t frames, uint64_t bins, const uint64_t* row_lens,
                            uint32_t sr, uint64_t k, float* out) {
    return probe_call([&]() -> int64_t {
        Spec m;
        spec_from_rows(spec, frames, bins, row_lens, &m);
        switch (kind) {
            case 0: return put_curve(spectral_flux_novelty(m), out);
            case 1: return put_curve(energy_flux_novelty(m), out);
            case 2: return put_curve(hfc_novelty(m, sr), out);
            default: return put_curve(superflux_novelty(m, (size_t)k), out);
        }
    });
}

// combined_novelty_with_params (novelty.rs:874-932); combined_novelty = (.5, .3, .2, 16, 5)
int64_t sdsp_oracle_combined_novelty(const float* s, uint64_t ns, const float* e, uint64_t ne, const float* h,
                                     uint64_t nh, float ws, float we, float wh, uint64_t lmw, uint64_t smw, float* out) {
    return probe_call([&]() -> int64_t {
        return put_curve(combined_novelty_params(std::vector<float>(s, s + ns), std::vector<float>(e, e + ne),
                                                 std::vector<float>(h, h + nh), ws, we, wh, (size_t)lmw, (size_t)smw),
                         out);
    });
}

// kind 0 fft_tempogram (tempogram_fft.rs:78-192), 1 autocorrelation_tempogram
// (tempogram_autocorr.rs:79-178): (bpm, value) pairs sorted by value, stable; returns the count
int64_t sdsp_oracle_tempogram(int32_t kind, const float* nov, uint64_t n, uint32_t sr, uint32_t hop, float min_bpm,
                              float max_bpm, float res, float* bpm, float* val, uint64_t cap) {
    return probe_call([&]() -> int64_t {
        const std::vector<float> v(nov, nov + n);
        const Tg tg = kind == 0 ? fft_tempogram(v, sr, hop, min_bpm, max_bpm) : acf_tempogram(v, sr, hop, min_bpm, max_bpm, res);
        for (size_t i = 0; i < tg.size() && i < cap; i++) {
            bpm[i] = tg[i].first;
            val[i] = tg[i].second;
        }
        return (int64_t)tg.size();
    });
}

// estimate_bpm_tempogram (tempogram.rs:155-174, no band fusion): out = (bpm, confidence, agreement)
int32_t sdsp_oracle_tempogram_estimate(const float* spec, uint64_t frames, uint64_t bins, uint32_t sr, uint32_t hop,
                                       float min_bpm, float max_bpm, float res, float* out3) {
    return (int32_t)probe_call([&]() -> int64_t {
        Spec m;
        spec_from_rows(spec, frames, bins, nullptr, &m);
        BpmEstimate e{};
        tempogram_impl(m, sr, hop, min_bpm, max_bpm, res, nullptr, &e, nullptr);
        out3[0] = e.bpm;
        out3[1] = e.confidence;
        out3[2] = (float)e.method_agreement;
        return 0;
    });
}

// multi_resolution_analysis (multi_resolution.rs:76-203): estimate_bpm_tempogram of the same
// spectrogram at hops 256/512/1024; all within 2 BPM -> mean BPM, mean conf x1.2 (<= 1),
// agreement = count; else the most confident (max_by: last maximum) with conf x0.9
int32_t sdsp_oracle_multi_resolution_analysis(const float* spec, uint64_t frames, uint64_t bins, uint32_t sr,
                                              float min_bpm, float max_bpm, float res, float* out3) {
    return (int32_t)probe_call([&]() -> int64_t {
        Spec m;
        spec_from_rows(spec, frames, bins, nullptr, &m);
        std::vector<BpmEstimate> rs;
        for (uint32_t hop : {256u, 512u, 1024u}) {
            try {
                BpmEstimate e{};
                tempogram_impl(m, sr, hop, min_bpm, max_bpm, res, nullptr, &e, nullptr);
                rs.push_back(e);
            } catch (const AErr&) {
            }
        }
        if (rs.empty()) fail(SDSP_ERR_PROCESSING, "All multi-resolution tempogram analyses failed");
        BpmEstimate r = rs[0];
        if (rs.size() >= 2) {
            bool agree = true;
            for (auto& e : rs) agree &= sd_absf(e.bpm - rs[0].bpm) < 2.0f;
            if (agree) {
                float sb = 0.0f, sc = 0.0f;
                for (auto& e : rs) sb += e.bpm;
                for (auto& e : rs) sc += e.confidence;
                r = {sb / (float)rs.size(), sd_minf((sc / (float)rs.size()) * 1.2f, 1.0f), (uint32_t)rs.size()};
            } else {
                size_t bi = 0;
                for (size_t i = 1; i < rs.size(); i++)
                    if (!(rs[i].confidence < rs[bi].confidence)) bi = i;
                r = {rs[bi].bpm, rs[bi].confidence * 0.9f, 1};
            }
        }
        out3[0] = r.bpm;
        out3[1] = r.confidence;
        out3[2] = (float)r.method_agreement;
        return 0;
    });
}
}
