// k_legacy.hip — the legacy BPM estimator (estimate_bpm / estimate_bpm_with_guardrails,
// reference src/features/period/mod.rs:196-404) for force_legacy_bpm and enable_bpm_fusion
// (src/lib.rs:294-329, 814-892).  One workgroup per track:
//
//   1. autocorrelation (autocorrelation.rs:90-268): the onset impulse train of length
//      L = max_onset / hop + 1, ACF by FFT of size M = next_pow2(2L) (sdsp_fft_spec.h, Stockham in
//      global scratch: M reaches 2^17 for 10-min tracks, beyond LDS), |X|^2, inverse, /M, max(0);
//      prominence peaks in the lag range (sequential, thread 0: the list is tiny).
//   2. comb filter (comb_filter.rs:96-215, 342-397): one thread per candidate BPM.  The reference
//      scans every onset for every expected beat (min_by_key of the truncated distance); on the
//      sorted onset list the first minimum is the nearer of the two onsets around the beat
//      (keys are monotone on either side), so each thread walks the beats with one moving index.
//      Normalised scores are sorted (confidence desc, BPM order on ties: the stable sort) by an
//      LDS bitonic sort; only the first 10 survive into the merge.
//   3. merge_bpm_candidates + consensus boost (candidate_filter.rs:40-442), guardrail multipliers
//      and the preferred-range promotion (mod.rs:88-121, 300-404): thread 0, the oracle's order.
//
// Arithmetic follows oracle/o_period.cpp operation for operation (f32, no contraction).
#include "../../include/sdsp_fft_spec.h"
#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdsp {

namespace {

constexpr int LG_T = 1024;

// Block-cooperative Stockham FFT over global memory, sdsp_fft_spec.h order.  tw is the Mt-point
// table read at stride Mt / M: tw_Mt[j * Mt / M] == tw_M[j] (both are cos/sin of the same double).
__device__ cx* lg_fft(cx* A, cx* B, int M, const cx* __restrict__ tw, int tws) {
    cx* src = A;
    cx* dst = B;
    int n = M, s = 1, ls = 0;
    while (n >= 4) {
        const int m = n >> 2, tstep = (M / n) * tws;
        for (int beta = threadIdx.x; beta < (M >> 2); beta += blockDim.x) {
            const int p = beta >> ls, q = beta & (s - 1);
            const cx a = src[q + s * p], b = src[q + s * (p + m)], c = src[q + s * (p + 2 * m)],
                     d = src[q + s * (p + 3 * m)];
            const cx w1 = tw[1 * p * tstep], w2 = tw[2 * p * tstep], w3 = tw[3 * p * tstep];
            const cx apc = cadd(a, c), amc = csub(a, c), bpd = cadd(b, d), bmd = csub(b, d);
            const cx jbmd = {bmd.im, -bmd.re};
            dst[q + s * (4 * p + 0)] = cadd(apc, bpd);
            dst[q + s * (4 * p + 1)] = cmul(w1, cadd(amc, jbmd));
            dst[q + s * (4 * p + 2)] = cmul(w2, csub(apc, bpd));
            dst[q + s * (4 * p + 3)] = cmul(w3, csub(amc, jbmd));
        }
        __syncthreads();
        cx* t = src;
        src = dst;
        dst = t;
        n = m;
        s <<= 2;
        ls += 2;
    }
    if (n == 2) {
        for (int q = threadIdx.x; q < s; q += blockDim.x) {
            const cx a = src[q], b = src[q + s];
            dst[q] = cadd(a, b);
            dst[q + s] = csub(a, b);
        }
        __syncthreads();
        cx* t = src;
        src = dst;
        dst = t;
    }
    return src;
}

struct Cand {
    float bpm, conf;
};
struct Est {
    float bpm, conf;
    uint32_t agree;
};

// Rust's stable sort on short slices == insertion sort (the oracle's insertion_sort).
template <class T, class Less>
__device__ void ins_sort(T* v, int n, Less less) {
    for (int i = 1; i < n; i++) {
        T tmp = v[i];
        int j = i;
        while (j > 0 && less(tmp, v[j - 1])) {
            v[j] = v[j - 1];
            j--;
        }
        v[j] = tmp;
    }
}

__device__ __forceinline__ uint64_t trunc_key(float d) { return sd_f2u64(d); }

// comb_filter.rs:342-397 on sorted onsets: aligned beats / expected beats.
__device__ float comb_score(const uint32_t* __restrict__ on, int n, uint32_t sr, float bpm, float tol) {
    const float period = (60.0f * (float)sr) / bpm;  // >= 1 (host-checked)
    const float tol_s = period * tol;
    const float last = (float)on[n - 1];
    const uint64_t nb = sd_f2u64(ceilf(last / period)) + 1;
    uint64_t aligned = 0;
    int idx = 0;  // first onset with (float)on >= e
    for (uint64_t bi = 0; bi < nb; bi++) {
        const float e = (float)bi * period;
        while (idx < n && (float)on[idx] < e) idx++;
        const uint64_t kl = idx > 0 ? trunc_key(sd_absf((float)on[idx - 1] - e)) : ~0ull;
        const uint64_t kr = idx < n ? trunc_key(sd_absf((float)on[idx] - e)) : ~0ull;
        int best;
        if (kl <= kr) {  // the first minimum lies left: walk back over equal keys
            best = idx - 1;
            while (best > 0 && trunc_key(sd_absf((float)on[best - 1] - e)) == kl) best--;
        } else {
            best = idx;
        }
        if (sd_absf((float)on[best] - e) <= tol_s) aligned++;
    }
    return nb > 0 ? (float)aligned / (float)nb : 0.0f;
}

__device__ __forceinline__ bool in_common(float b) { return b >= 60.0f && b <= 180.0f; }

}  // namespace

__global__ __launch_bounds__(LG_T) void k_legacy(const uint32_t* __restrict__ onsets, const uint64_t* __restrict__ on_off,
                                                 const int* __restrict__ on_n, int n_items,
                                                 const uint64_t* __restrict__ scr_off, const uint64_t* __restrict__ scr_cap,
                                                 cx* __restrict__ scratch, const cx* __restrict__ tw, int tw_M,
                                                 LegacyParams P, LegacyOut* __restrict__ out) {
    __shared__ float c_bpm[LG_COMB_MAX];
    __shared__ float c_sc[LG_COMB_MAX];
    __shared__ uint64_t c_key[LG_COMB_MAX];
    __shared__ uint32_t pk_lag[LG_AC_MAX];
    __shared__ float pk_val[LG_AC_MAX];
    __shared__ Cand ac[LG_AC_MAX];
    __shared__ Cand al[LG_AC_MAX + 10];
    __shared__ Cand cl[10];
    __shared__ Est est[LG_AC_MAX + 20];
    __shared__ float gb_total[LG_AC_MAX + 20], gb_maxc[LG_AC_MAX + 20];
    __shared__ float red[LG_T / 64];
    __shared__ int sh_i[4];
    const int t = blockIdx.x;
    if (t >= n_items) return;
    const int n = on_n[t];
    const uint32_t* on = onsets + on_off[t];
    if (n < 2) {  // on_legacy.len() < 2 -> no legacy estimate (src/lib.rs:296)
        if (threadIdx.x == 0) out[t] = LegacyOut{0, 0.0f, 0.0f, 0};
        return;
    }
    // ---------------- 1. autocorrelation ----------------
    const uint64_t L = (uint64_t)on[n - 1] / (uint64_t)P.hop + 1;  // sorted: the last onset is the max
    if (L < 2) {  // "Signal too short for autocorrelation" (autocorrelation.rs:128-133) propagates
        if (threadIdx.x == 0) out[t] = LegacyOut{-1, 0.0f, 0.0f, 0};
        return;
    }
    int M = 1;
    while ((uint64_t)M < 2 * L) M <<= 1;
    if ((uint64_t)M > scr_cap[t] || M > tw_M) {
        if (threadIdx.x == 0) out[t] = LegacyOut{-2, 0.0f, 0.0f, 0};
        return;
    }
    cx* A = scratch + scr_off[t];
    cx* B = A + scr_cap[t];
    for (int i = threadIdx.x; i < M; i += blockDim.x) A[i] = cx{0.0f, 0.0f};
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += blockDim.x) A[on[k] / (uint32_t)P.hop] = cx{1.0f, 0.0f};
    __syncthreads();
    cx* X = lg_fft(A, B, M, tw, tw_M / M);
    for (int i = threadIdx.x; i < M; i += blockDim.x) {  // X *= conj(X); conj for the inverse
        const cx c = X[i];
        const float re = c.re * c.re - c.im * (-c.im);
        const float im = c.re * (-c.im) + c.im * c.re;
        X[i] = cx{re, -im};
    }
    __syncthreads();
    cx* Y = lg_fft(X, X == A ? B : A, M, tw, tw_M / M);
    float* acf = reinterpret_cast<float*>(Y == A ? B : A);  // the free buffer holds the ACF
    const float scale = 1.0f / (float)M;
    float mloc = 0.0f;
    for (uint64_t i = threadIdx.x; i < L; i += blockDim.x) {
        const float v = sd_maxf(Y[i].re * scale, 0.0f);
        acf[i] = v;
        mloc = sd_maxf(mloc, v);
    }
    const float max_acf = block_max(mloc, red);  // also the barrier before thread 0 reads acf
    const uint64_t lag_min = sd_f2u64(ceilf((60.0f * (float)P.sr) / (P.max_bpm * (float)P.hop)));
    const uint64_t lag_max = sd_f2u64(floorf((60.0f * (float)P.sr) / (P.min_bpm * (float)P.hop)));
    if (threadIdx.x == 0) {
        int nac = 0;
        if (!(lag_min >= lag_max || lag_min >= L || lag_max >= L)) {
            // find_peaks_in_acf (autocorrelation.rs:280-338)
            const float* a = acf + lag_min;
            const uint64_t len = lag_max - lag_min + 1;
            float mx = 0.0f;
            for (uint64_t i = 0; i < len; i++) mx = sd_maxf(mx, a[i]);
            int np = 0;
            if (!(mx < EPS)) {
                const float min_prom = mx * 0.1f;
                for (uint64_t i = 1; i + 1 < len; i++) {
                    const float v = a[i];
                    if (v > a[i - 1] && v > a[i + 1]) {
                        const float prom = v - sd_maxf(a[i - 1], a[i + 1]);
                        if (prom >= min_prom) {
                            const uint32_t lag = (uint32_t)(i + lag_min);
                            const int64_t dl = (int64_t)(int32_t)lag - (int64_t)(int32_t)(np ? pk_lag[np - 1] : 0u);
                            if (np == 0 || (dl < 0 ? -dl : dl) >= 2) {
                                if (np < LG_AC_MAX) {
                                    pk_lag[np] = lag;
                                    pk_val[np] = v;
                                    np++;
                                }
                            } else if (v > pk_val[np - 1]) {
                                pk_lag[np - 1] = lag;
                                pk_val[np - 1] = v;
                            }
                        }
                    }
                }
            }
            for (int i = 0; i < np; i++) {  // (lag, value) pairs as candidates, sorted by value desc
                ac[i].bpm = (float)pk_lag[i];
                ac[i].conf = pk_val[i];
            }
            ins_sort(ac, np, [](const Cand& x, const Cand& y) { return y.conf < x.conf; });
            for (int i = 0; i < np; i++) {
                const float lagf = ac[i].bpm;
                const float bpm = (60.0f * (float)P.sr) / (lagf * (float)P.hop);
                if (bpm >= P.min_bpm && bpm <= P.max_bpm) {
                    const float conf = max_acf > EPS ? sd_minf(ac[i].conf / max_acf, 1.0f) : 0.0f;
                    ac[nac++] = Cand{bpm, conf};
                }
            }
            ins_sort(ac, nac, [](const Cand& x, const Cand& y) { return y.conf < x.conf; });
        }
        sh_i[0] = nac;
        // candidate BPMs of the comb filter: bpm = min; bpm <= max + EPS; bpm += res (f32)
        int nc = 0;
        for (float bpm = P.min_bpm; bpm <= P.max_bpm + EPS && nc < LG_COMB_MAX; bpm += P.res) c_bpm[nc++] = bpm;
        sh_i[1] = nc;
    }
    __syncthreads();
    const int nac = sh_i[0], nc = sh_i[1];
    // ---------------- 2. comb filter ----------------
    float smax = 0.0f;
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        const float bpm = c_bpm[i];
        const float at = sd_clampf(0.1f * (120.0f / bpm), 0.05f, 0.15f);
        const float sc = comb_score(on, n, (uint32_t)P.sr, bpm, at);
        c_sc[i] = sc;
        smax = sd_maxf(smax, sc);
    }
    const float max_score = block_max(smax, red);
    int np2 = 1;
    while (np2 < nc) np2 <<= 1;
    for (int i = threadIdx.x; i < np2; i += blockDim.x) {
        if (i < nc) {
            const float conf = max_score > EPS ? c_sc[i] / max_score : 0.0f;
            c_sc[i] = conf;
            c_key[i] = key_desc_nonneg(conf, (uint32_t)i);
        } else {
            c_key[i] = ~0ull;
        }
    }
    block_bitonic_u64(c_key, np2);
    // ---------------- 3. merge, boost, guardrails (thread 0) ----------------
    if (threadIdx.x != 0) return;
    int ncomb = 0;  // retain(conf >= 0.1): a prefix of the sorted list; only the first 10 are read
    for (int i = 0; i < nc && ncomb < 10; i++) {
        const uint32_t j = (uint32_t)(c_key[i] & 0xffffffffu);
        if (!(c_sc[j] >= 0.1f)) break;
        cl[ncomb++] = Cand{c_bpm[j], c_sc[j]};
    }
    // preferred-range top autocorr BPM (mod.rs:312-325), before the merge rewrites the list
    const float pmin = P.guard ? P.g[0] : 60.0f, pmax = P.guard ? P.g[1] : 180.0f;
    bool have_top = false;
    float top_pref = 0.0f;
    for (int i = 0; i < nac; i++)
        if (ac[i].bpm >= pmin && ac[i].bpm <= pmax) {
            have_top = true;
            top_pref = ac[i].bpm;
            break;
        }
    if (nac == 0 && ncomb == 0) {
        out[t] = LegacyOut{0, 0.0f, 0.0f, 0};
        return;
    }
    // merge_bpm_candidates (candidate_filter.rs:147-442), ac modified in place (it is a copy)
    const float tol_ratio = sd_exp2f(50.0f / 1200.0f);
    const int n3 = ncomb < 3 ? ncomb : 3;
    for (int k = 0; k < nac; k++) {
        for (int i = 0; i < n3; i++) {
            const float ratio = ac[k].bpm / cl[i].bpm;
            const float rt = ratio / 2.0f;
            if (sd_absf(rt - 1.0f) < (tol_ratio - 1.0f)) {
                const bool corr = in_common(cl[i].bpm) || (ac[k].bpm > 200.0f || ac[k].bpm < 30.0f);
                if (corr) {
                    ac[k].bpm = cl[i].bpm;
                    break;
                }
            }
        }
    }
    for (int k = 0; k < nac; k++) {
        for (int i = 0; i < n3; i++) {
            const float ratio = cl[i].bpm / ac[k].bpm;
            const float rt = ratio / 2.0f;
            if (sd_absf(rt - 1.0f) < (tol_ratio - 1.0f)) {
                if (in_common(cl[i].bpm)) {
                    ac[k].bpm = cl[i].bpm;
                    break;
                }
            }
        }
    }
    bool disagree = false;
    if (nac > 0 && ncomb > 0) {
        const float d = sd_absf(ac[0].bpm - cl[0].bpm);
        disagree = d > 10.0f && d < 50.0f;
    }
    int nal = nac < 10 ? nac : 10;
    for (int i = 0; i < nal; i++) al[i] = ac[i];
    for (int k = 0; k < nac; k++) {
        if (in_common(ac[k].bpm)) {
            bool near = false;
            for (int i = 0; i < nal; i++) near |= sd_absf(al[i].bpm - ac[k].bpm) < 1.0f;
            if (!near && nal < LG_AC_MAX + 10) al[nal++] = ac[k];
        }
    }
    int ng = 0;
    auto add = [&](const Cand& c) {
        for (int g = 0; g < ng; g++) {
            if (sd_absf(c.bpm - est[g].bpm) <= 2.0f) {
                const uint32_t cnt = est[g].agree;
                est[g].bpm = (est[g].bpm * (float)cnt + c.bpm) / (float)(cnt + 1);
                gb_total[g] += c.conf;
                est[g].agree += 1;
                gb_maxc[g] = sd_maxf(gb_maxc[g], c.conf);
                return;
            }
        }
        est[ng] = Est{c.bpm, 0.0f, 1};
        gb_total[ng] = c.conf;
        gb_maxc[ng] = c.conf;
        ng++;
    };
    for (int i = 0; i < nal; i++) add(al[i]);
    for (int i = 0; i < ncomb; i++) add(cl[i]);
    for (int g = 0; g < ng; g++) {
        float conf;
        if (est[g].agree >= 2) {
            const float avg = gb_total[g] / (float)est[g].agree;
            conf = sd_minf((avg + gb_maxc[g]) / 2.0f * 1.2f, 1.0f);
        } else {
            conf = sd_minf(gb_total[g], 1.0f);
        }
        if (disagree && est[g].agree == 1) conf *= 0.7f;
        est[g].conf = conf;
    }
    // boost_consensus (candidate_filter.rs:40-97) against the first 5 of each list
    const int a5 = nal < 5 ? nal : 5, c5 = ncomb < 5 ? ncomb : 5;
    for (int g = 0; g < ng; g++) {
        Est& e = est[g];
        bool ad = false, cd = false, ah = false, ch = false;
        for (int i = 0; i < a5; i++) ad |= sd_absf(al[i].bpm - e.bpm) < 2.5f;
        for (int i = 0; i < c5; i++) cd |= sd_absf(cl[i].bpm - e.bpm) < 2.5f;
        for (int i = 0; i < a5; i++) {
            const float r = sd_maxf(al[i].bpm / e.bpm, e.bpm / al[i].bpm);
            ah |= sd_absf(r - 2.0f) < 0.1f || sd_absf(r - 1.5f) < 0.1f || sd_absf(r - 0.75f) < 0.1f;
        }
        for (int i = 0; i < c5; i++) {
            const float r = sd_maxf(cl[i].bpm / e.bpm, e.bpm / cl[i].bpm);
            ch |= sd_absf(r - 2.0f) < 0.1f || sd_absf(r - 1.5f) < 0.1f || sd_absf(r - 0.75f) < 0.1f;
        }
        if (ad && cd)
            e.conf *= 1.5f;
        else if ((ad && ch) || (cd && ah))
            e.conf *= 1.3f;
        if (cd && e.bpm >= 60.0f && e.bpm <= 180.0f) e.conf *= 1.4f;
    }
    bool reasonable5 = false;
    for (int g = 0; g < ng && g < 5; g++) reasonable5 |= in_common(est[g].bpm);
    if (!reasonable5) {
        for (int g = 0; g < ng; g++)
            if (in_common(est[g].bpm)) {
                est[g].conf *= 2.0f;
                break;
            }
    }
    ins_sort(est, ng, [](const Est& a, const Est& b) {
        const bool ai = in_common(a.bpm), bi = in_common(b.bpm);
        const float ae = ai ? a.conf : a.conf * 0.5f;
        const float be = bi ? b.conf : b.conf * 0.5f;
        int ec = (be < ae) ? -1 : (be > ae) ? 1 : 0;
        if (sd_absf(ae - be) < 0.5f) {
            if (ai && !bi) return true;
            if (!ai && bi) return false;
        }
        if (ec != 0) return ec < 0;
        return b.agree < a.agree;
    });
    // guardrails (mod.rs:300-360): confidence multipliers by range, stable re-sort
    if (P.guard) {
        for (int g = 0; g < ng; g++) {
            Est& e = est[g];
            float mul;
            if (!sd_isfinite_f(e.bpm))
                mul = 0.0f;
            else if (e.bpm >= P.g[0] && e.bpm <= P.g[1])
                mul = P.g[4];
            else if (e.bpm >= P.g[2] && e.bpm <= P.g[3])
                mul = P.g[5];
            else
                mul = P.g[6];
            e.conf *= mul;
        }
        ins_sort(est, ng, [](const Est& a, const Est& b) { return b.conf < a.conf; });
    }
    int first = 0;
    if (have_top) {  // move the first estimate near the preferred autocorr BPM to the front
        for (int g = 0; g < ng; g++)
            if (sd_absf(est[g].bpm - top_pref) < 2.0f) {
                first = g;
                break;
            }
    }
    if (ng == 0) {
        out[t] = LegacyOut{0, 0.0f, 0.0f, 0};
        return;
    }
    out[t] = LegacyOut{1, est[first].bpm, est[first].conf, (int)est[first].agree};
}

void launch_legacy(const uint32_t* onsets, const uint64_t* on_off, const int* on_n, int n_items, const uint64_t* scr_off,
                   const uint64_t* scr_cap, cx* scratch, const cx* tw, int tw_M, const LegacyParams& P, LegacyOut* out,
                   hipStream_t st) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_legacy, dim3((unsigned)n_items), dim3(LG_T), 0, st, onsets, on_off, on_n, n_items, scr_off,
                       scr_cap, scratch, tw, tw_M, P, out);
}

}  // namespace sdsp
