// k_tempo.hip — tempogram kernels.
//
//   k_fft_tempogram    fft_tempogram + find_best_bpm_fft      src/features/period/tempogram_fft.rs:78-236
//   k_acf_tempogram    autocorrelation_tempogram              tempogram_autocorr.rs:79-178
//   k_tempo_select     estimate_bpm_tempogram_impl scoring    tempogram.rs:501-775 (+ gate src/lib.rs:410-459)
//   k_multires         multi_resolution fusion / folds        multi_resolution.rs:272-901
//
// Work lists: every launch takes an explicit list of (track, variant) items so the same
// kernels serve the base pass (hop 512, all tracks) and the escalation pass (hops 256/1024,
// only the tracks whose base estimate is ambiguous).
#include "../../include/sdsp_fft_spec.h"
#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdsp {

constexpr int NACF_MAX = 512;
constexpr int ACF_U = 16;  // k_acf_tempogram: fold steps loaded per block
constexpr int ACF_CH = 4096;   // k_acf_tempogram: frames per LDS chunk
constexpr int ACF_HMAX = 1024; // k_acf_tempogram: the largest lag the LDS path serves (its halo)

// ----------------------------------------------------------------------------------------
// Block-cooperative complex FFT, Stockham radix-4 (+radix-2) exactly as sdsp_fft_spec.h.
// A holds the input; returns the buffer holding the output (A or B).
__device__ cx* fft_block(cx* A, cx* B, int M, const cx* __restrict__ tw) {
    cx* src = A;
    cx* dst = B;
    int n = M, s = 1, ls = 0;
    while (n >= 4) {
        const int m = n >> 2, tstep = M / n;
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

// In-place variant for a single LDS buffer (M <= 4 * 256 * RMAX): each radix-4 pass reads
// its butterflies' inputs into registers, barriers, then writes the outputs -- the same
// arithmetic and output positions as fft_block with half the LDS, so an FFT tempogram block
// fits on a CU beside the STFT blocks of the other stream.
template <int RMAX>
__device__ cx* fft_block_inplace(cx* A, int M, const cx* __restrict__ tw) {
    int n = M, s = 1, ls = 0;
    const int nb = M >> 2;
    while (n >= 4) {
        const int m = n >> 2, tstep = M / n;
        cx o[RMAX][4];
        int ob[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; r++) {
            const int beta = threadIdx.x + r * blockDim.x;
            ob[r] = -1;
            if (beta < nb) {
                const int p = beta >> ls, q = beta & (s - 1);
                const cx a = A[q + s * p], b = A[q + s * (p + m)], c = A[q + s * (p + 2 * m)],
                         d = A[q + s * (p + 3 * m)];
                const cx w1 = tw[1 * p * tstep], w2 = tw[2 * p * tstep], w3 = tw[3 * p * tstep];
                const cx apc = cadd(a, c), amc = csub(a, c), bpd = cadd(b, d), bmd = csub(b, d);
                const cx jbmd = {bmd.im, -bmd.re};
                o[r][0] = cadd(apc, bpd);
                o[r][1] = cmul(w1, cadd(amc, jbmd));
                o[r][2] = cmul(w2, csub(apc, bpd));
                o[r][3] = cmul(w3, csub(amc, jbmd));
                ob[r] = q + s * 4 * p;
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RMAX; r++)
            if (ob[r] >= 0) {
                A[ob[r]] = o[r][0];
                A[ob[r] + s] = o[r][1];
                A[ob[r] + 2 * s] = o[r][2];
                A[ob[r] + 3 * s] = o[r][3];
            }
        __syncthreads();
        n = m;
        s <<= 2;
        ls += 2;
    }
    if (n == 2) {  // each thread reads and writes the same two slots
        for (int q = threadIdx.x; q < s; q += blockDim.x) {
            const cx a = A[q], b = A[q + s];
            A[q] = cadd(a, b);
            A[q + s] = csub(a, b);
        }
        __syncthreads();
    }
    return A;
}
constexpr int FFT_TG_RMAX = 8;  // in-place LDS FFT up to M = 8192 (P = 16384)

// ----------------------------------------------------------------------------------------
// FFT tempogram.  items[i] = trk*NVAR + v.  Output entries for item i at out_off[i], count K.
// LDS: the in-place LDS FFT (P.lds); otherwise the Stockham ping-pong through L2-resident global
// scratch, instantiated as its own kernel so it carries none of the in-place FFT's registers.
template <bool LDS>
__global__ __launch_bounds__(256) void k_fft_tempogram(const int* __restrict__ items, int n_items, int T,
                                                       const float* __restrict__ nov, const float* __restrict__ nov_sum,
                                                       const uint64_t* __restrict__ frame_pfx, uint64_t total,
                                                       FftTgParams P, const cx* __restrict__ tw,
                                                       const cx* __restrict__ rt, cx* __restrict__ gscratch,
                                                       const uint64_t* __restrict__ out_off, float* __restrict__ out_bpm,
                                                       float* __restrict__ out_pow) {
    SDSP_LATENCY_CRITICAL();
    extern __shared__ cx dyn[];
    const int it = items[blockIdx.x];
    const int trk = it / NVAR, v = it % NVAR;
    const int64_t L = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]) - 1;
    const float* x = nov + (uint64_t)v * total + frame_pfx[trk];
    const int M = P.P / 2;
    cx* A;
    cx* Bb;
    if constexpr (LDS) {
        A = dyn;
        Bb = dyn + M;
    } else {
        A = gscratch + (uint64_t)blockIdx.x * 2 * (uint64_t)M;
        Bb = A + M;
    }
    const float mean = nov_sum[(uint64_t)v * T + trk] / (float)L;
    const int n = (int)L;
    for (int j = threadIdx.x; j < M; j += blockDim.x) {
        float r0 = 0.0f, r1 = 0.0f;
        const int i0 = 2 * j, i1 = 2 * j + 1;
        if (i0 < n) r0 = (x[i0] - mean) * (n > 1 ? sdsp_hann_f32(i0, n) : 1.0f);
        if (i1 < n) r1 = (x[i1] - mean) * (n > 1 ? sdsp_hann_f32(i1, n) : 1.0f);
        A[j] = {r0, r1};
    }
    __syncthreads();
    cx* Z;
    uint64_t* keys;
    if constexpr (LDS) {  // one M-slot buffer + the key buffer (dyn[M ..])
        Z = (M >= 2) ? fft_block_inplace<FFT_TG_RMAX>(A, M, tw) : A;
        keys = reinterpret_cast<uint64_t*>(dyn + M);
    } else {
        Z = (M >= 2) ? fft_block(A, Bb, M, tw) : A;
        keys = reinterpret_cast<uint64_t*>((Z == A) ? Bb : A);
    }
    int K2 = 1;
    while (K2 < P.K) K2 <<= 1;
    for (int i = threadIdx.x; i < K2; i += blockDim.x) {
        uint64_t key = ~0ull;
        if (i < P.K) {
            const int k = P.b_lo + i;
            float pw;
            if (M >= 1) {
                const cx Zk = Z[k & (M - 1)];
                const cx Zr = Z[(M - k) & (M - 1)];
                const cx Zc = {Zr.re, -Zr.im};
                const cx E = {(Zk.re + Zc.re) * 0.5f, (Zk.im + Zc.im) * 0.5f};
                const cx D = csub(Zk, Zc);
                const cx O = {D.im * 0.5f, -(D.re * 0.5f)};
                const cx X = cadd(E, cmul(rt[k], O));
                pw = X.re * X.re + X.im * X.im;
            } else {
                pw = 0.0f;
            }
            key = key_desc(pw, (uint32_t)i);
        }
        keys[i] = key;
    }
    // keys live in the buffer the FFT result is not in: the reads of Z above are complete
    // for every thread only after the barrier inside the sort's first step.
    block_bitonic_u64(keys, K2);
    float* ob = out_bpm + out_off[blockIdx.x];
    float* op = out_pow + out_off[blockIdx.x];
    for (int i = threadIdx.x; i < P.K; i += blockDim.x) {
        const uint64_t key = keys[i];
        const int idx = (int)(key & 0xffffffffu);
        const uint32_t ou = ~(uint32_t)(key >> 32);
        const uint32_t u = (ou & 0x80000000u) ? (ou & 0x7fffffffu) : ~ou;  // inverse of ord_f
        ob[i] = (float)(P.b_lo + idx) * P.fres * 60.0f;
        op[i] = sd_from_bits_f(u);
    }
}

// ----------------------------------------------------------------------------------------
// Autocorrelation tempogram: one thread per BPM of the min..=max grid (lag per BPM given).  The
// lag sum is a sequential fold; its operands are loaded ACF_U steps at a time, the next block in
// flight while the current one is folded, so the fold waits on one L2 round trip per ACF_U steps
// instead of one per step.  (Staging the curve in LDS measured 2x slower: 62 KB per workgroup
// cut the waves per CU.)
__global__ __launch_bounds__(256) void k_acf_tempogram(const int* __restrict__ items, const float* __restrict__ nov,
                                                       const uint64_t* __restrict__ frame_pfx, uint64_t total,
                                                       const float* __restrict__ bpm_grid,
                                                       const int* __restrict__ lag_grid, int NB,
                                                       float* __restrict__ out_bpm, float* __restrict__ out_str) {
    SDSP_LATENCY_CRITICAL();
    __shared__ uint64_t keys[NACF_MAX];
    __shared__ float vals[NACF_MAX];
    const int it = items[blockIdx.x];
    const int trk = it / NVAR, v = it % NVAR;
    const int64_t L = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]) - 1;
    const float* x = nov + (uint64_t)v * total + frame_pfx[trk];
    int K2 = 1;
    while (K2 < NB) K2 <<= 1;
#ifndef SDSP_ACF_GLOBAL
    // The novelty is staged through LDS in ACF_CH-frame chunks with the largest lag as halo, and
    // every lag's thread continues its fold across the chunks (i ascending, the same products in
    // the same order): each step reads LDS instead of two vector-memory loads per element, which
    // held the kernel at the texture unit's address rate.  Lags beyond the halo keep the global path.
    __shared__ float xs[ACF_CH + ACF_HMAX];
    __shared__ int lagmax_s;
    if (threadIdx.x == 0) lagmax_s = 0;
    __syncthreads();
    int lm = 0;
    for (int j = threadIdx.x; j < NB; j += blockDim.x) lm = max(lm, lag_grid[j]);
    atomicMax(&lagmax_s, lm);
    __syncthreads();
    const int lagmax = lagmax_s;
    if (NB <= (int)blockDim.x && lagmax >= 0 && lagmax <= ACF_HMAX) {
        const int j = threadIdx.x;
        const int64_t lag = j < NB ? lag_grid[j] : 0;
        const int64_t n = j < NB ? L - lag : 0;  // terms i = 0 .. n-1
        float acc = 0.0f;
        for (int64_t c0 = 0; c0 < L; c0 += ACF_CH) {
            const int64_t m = L - c0 < ACF_CH + lagmax ? L - c0 : ACF_CH + lagmax;  // x[c0 .. c0+m) staged
            __syncthreads();  // the previous chunk's reads are done
            for (int k = threadIdx.x; k < m; k += blockDim.x) xs[k] = x[c0 + k];
            __syncthreads();
            const int64_t e = n < c0 + ACF_CH ? n : c0 + ACF_CH;  // this chunk's terms: i in [c0, e)
            const int cnt = e > c0 ? (int)(e - c0) : 0;
            const float* xl = xs + lag;
#pragma unroll 8
            for (int i = 0; i < cnt; i++) acc += xs[i] * xl[i];
        }
        if (j < NB) {
            const int32_t cnt = n > 0 ? (int32_t)n : 0;
            const float sv = cnt > 0 ? acc / (float)cnt : 0.0f;
            vals[j] = sv;
            keys[j] = key_desc(sv, (uint32_t)j);
        } else if (j < K2) {
            keys[j] = ~0ull;  // K2 <= blockDim.x here (NB <= blockDim.x)
        }
    } else
#endif
    for (int j = threadIdx.x; j < K2; j += blockDim.x) {
        uint64_t key = ~0ull;
        if (j < NB) {
            const int64_t lag = lag_grid[j];
            const int64_t n = L - lag;  // terms i = 0 .. n-1 (autocorrelation over i + lag < L)
            float acc = 0.0f;
            int64_t i = 0;
            if (n >= ACF_U) {
                float a[ACF_U], b[ACF_U], na[ACF_U], nb[ACF_U];
#pragma unroll
                for (int u = 0; u < ACF_U; u++) {
                    a[u] = x[u];
                    b[u] = x[u + lag];
                }
                for (;;) {
                    const bool more = i + 2 * ACF_U <= n;
                    if (more) {
#pragma unroll
                        for (int u = 0; u < ACF_U; u++) {
                            na[u] = x[i + ACF_U + u];
                            nb[u] = x[i + ACF_U + u + lag];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < ACF_U; u++) acc += a[u] * b[u];
                    i += ACF_U;
                    if (!more) break;
#pragma unroll
                    for (int u = 0; u < ACF_U; u++) {
                        a[u] = na[u];
                        b[u] = nb[u];
                    }
                }
            }
            for (; i < n; i++) acc += x[i] * x[i + lag];
            const int32_t cnt = n > 0 ? (int32_t)n : 0;
            const float sv = cnt > 0 ? acc / (float)cnt : 0.0f;
            vals[j] = sv;
            key = key_desc(sv, (uint32_t)j);
        }
        keys[j] = key;
    }
    block_bitonic_u64(keys, K2);
    float* ob = out_bpm + (uint64_t)blockIdx.x * NB;
    float* os = out_str + (uint64_t)blockIdx.x * NB;
    for (int i = threadIdx.x; i < NB; i += blockDim.x) {
        const int j = (int)(keys[i] & 0xffffffffu);
        ob[i] = bpm_grid[j];
        os[i] = vals[j];
    }
}

// ----------------------------------------------------------------------------------------
// Candidate generation + scoring (estimate_bpm_tempogram_impl, tempogram.rs:501-775).
__device__ float lookup_nearest(const float* bpm, const float* val, int n, float q, float tol) {
    float bd = SD_INF_F, bv = 0.0f;
    for (int i = 0; i < n; i++) {
        const float d = sd_absf(bpm[i] - q);
        if (d <= tol && d < bd) {
            bd = d;
            bv = val[i];
        }
    }
    return bv;
}

constexpr int SEL_MAXC = 1024;

__global__ __launch_bounds__(256) void k_tempo_select(const int* __restrict__ active, int n_items,
                                                      const float* __restrict__ fft_bpm,
                                                      const float* __restrict__ fft_pow,
                                                      const uint64_t* __restrict__ fft_off,  // per item*NVAR+v
                                                      const int* __restrict__ fft_k,         // per item
                                                      const float* __restrict__ acf_bpm,
                                                      const float* __restrict__ acf_str,
                                                      const uint64_t* __restrict__ acf_off,  // per item*NVAR+v
                                                      SelParams P, TempoEst* __restrict__ est,
                                                      float* __restrict__ cand, int cand_cap) {
    SDSP_LATENCY_CRITICAL();
    __shared__ uint64_t keys[SEL_MAXC];
    __shared__ float cvals[SEL_MAXC];
    __shared__ float sc[SEL_MAXC][3];  // score, fft_norm, ac_norm (indexed by uniq position)
    __shared__ int n_uniq_s, n_c_s;
    __shared__ float maxf[NVAR], maxa[NVAR];
    const int item = blockIdx.x;
    if (!active[item]) {  // fewer than 2 frames: "Novelty curve is empty after extraction"
        if (threadIdx.x == 0) est[item] = TempoEst{0.0f, 0.0f, 0, 0, 0, 0, 0, 0};
        return;
    }
    const int Kf = fft_k[item];
    const int NB = P.NB;
    const float* fb[NVAR];
    const float* fp[NVAR];
    const float* ab[NVAR];
    const float* as[NVAR];
    for (int v = 0; v < NVAR; v++) {
        fb[v] = fft_bpm + fft_off[item * NVAR + v];
        fp[v] = fft_pow + fft_off[item * NVAR + v];
        ab[v] = acf_bpm + acf_off[item * NVAR + v];
        as[v] = acf_str + acf_off[item * NVAR + v];
    }
    if (threadIdx.x < NVAR) {
        const int v = threadIdx.x;
        maxf[v] = sd_maxf(Kf > 0 ? fp[v][0] : 1.0f, 1e-12f);
        maxa[v] = sd_maxf(NB > 0 ? as[v][0] : 1.0f, 1e-12f);
    }
    const float fft_pb = Kf > 0 ? fb[0][0] : 0.0f;
    const float ac_pb = NB > 0 ? ab[0][0] : 0.0f;
    // seeds -> candidates (tempogram.rs:538-558)
    if (threadIdx.x == 0) {
        const float FACT[7] = {1.0f, 0.5f, 2.0f, 1.0f / 3.0f, 3.0f, 2.0f / 3.0f, 3.0f / 2.0f};
        int nc = 0;
        auto push_seed = [&](float b) {
            for (int k = 0; k < 7; k++) {
                const float x = b * FACT[k];
                if (sd_isfinite_f(x) && x >= P.min_bpm && x <= P.max_bpm && nc < SEL_MAXC) cvals[nc++] = x;
            }
        };
        for (int v = 0; v < NVAR; v++) {
            if (!P.present[v]) continue;
            for (int i = 0; i < 8 && i < Kf; i++) push_seed(fb[v][i]);
            for (int i = 0; i < 8 && i < NB; i++) push_seed(ab[v][i]);
        }
        if (fft_pb > 0.0f) push_seed(fft_pb);
        if (ac_pb > 0.0f) push_seed(ac_pb);
        n_c_s = nc;
    }
    __syncthreads();
    const int nc = n_c_s;
    for (int i = threadIdx.x; i < SEL_MAXC; i += blockDim.x) keys[i] = i < nc ? key_asc(cvals[i], (uint32_t)i) : ~0ull;
    block_bitonic_u64(keys, SEL_MAXC);
    __shared__ float uniq[SEL_MAXC];
    if (threadIdx.x == 0) {
        int nu = 0;
        for (int i = 0; i < nc; i++) {
            const float b = cvals[keys[i] & 0xffffffffu];
            if (nu > 0 && sd_absf(b - uniq[nu - 1]) < 0.75f) continue;
            uniq[nu++] = b;
        }
        n_uniq_s = nu;
    }
    __syncthreads();
    const int nu = n_uniq_s;
    float w_sum = 0.0f;
    for (int v = 0; v < NVAR; v++)
        if (P.present[v] && (!P.seed_only || v == 0)) w_sum += sd_maxf(P.w[v], 0.0f);
    w_sum = sd_maxf(w_sum, 1e-6f);
    for (int u = threadIdx.x; u < nu; u += blockDim.x) {
        const float bpm = uniq[u];
        float fa = 0.0f, aa = 0.0f;
        for (int v = 0; v < NVAR; v++) {
            if (!P.present[v] || (P.seed_only && v != 0)) continue;
            if (P.w[v] <= 0.0f) continue;
            const float fv = lookup_nearest(fb[v], fp[v], Kf, bpm, 0.75f);
            const float av = lookup_nearest(ab[v], as[v], NB, bpm, P.ac_tol);
            fa += P.w[v] * sd_clampf(fv / maxf[v], 0.0f, 1.0f);
            aa += P.w[v] * sd_clampf(av / maxa[v], 0.0f, 1.0f);
        }
        const float fn = sd_clampf(fa / w_sum, 0.0f, 1.0f);
        const float an = sd_clampf(aa / w_sum, 0.0f, 1.0f);
        float score = 0.55f * an + 0.45f * fn;
        if (P.bonus_on) {
            uint32_t sb = 0;
            for (int v = 1; v < NVAR; v++) {
                if (!P.present[v]) continue;
                const float sf = sd_clampf(lookup_nearest(fb[v], fp[v], Kf, bpm, 0.75f) / maxf[v], 0.0f, 1.0f);
                const float sa = sd_clampf(lookup_nearest(ab[v], as[v], NB, bpm, P.ac_tol) / maxa[v], 0.0f, 1.0f);
                if (sd_maxf(sf, sa) >= P.support_thr) sb++;
            }
            if (sb >= 2) score *= 1.0f + P.bonus * ((float)sb - 1.0f);
        }
        if (bpm > 180.0f)
            score *= 0.80f;
        else if (bpm < 60.0f)
            score *= 0.90f;
        sc[u][0] = score;
        sc[u][1] = fn;
        sc[u][2] = an;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SEL_MAXC; i += blockDim.x) keys[i] = i < nu ? key_desc(sc[i][0], (uint32_t)i) : ~0ull;
    block_bitonic_u64(keys, SEL_MAXC);
    if (threadIdx.x == 0) {
        TempoEst r{};
        if (nu == 0) {
            r.ok = 0;  // "No BPM candidates could be scored"
            est[item] = r;
        } else {
            int bi = (int)(keys[0] & 0xffffffffu);
            float bb = uniq[bi], bs = sc[bi][0], bfn = sc[bi][1], ban = sc[bi][2];
            if (bb > 180.0f) {  // tempo-octave fold (tempogram.rs:669-699)
                const float folded = bb / 2.0f;
                if (folded >= P.min_bpm && folded <= P.max_bpm) {
                    for (int k = 0; k < nu; k++) {
                        const int ci = (int)(keys[k] & 0xffffffffu);
                        if (sd_absf(uniq[ci] - folded) < 0.75f) {
                            const float eps = 1e-6f;
                            const float ar = (ban + eps) / (sc[ci][2] + eps);
                            const float fr = (bfn + eps) / (sc[ci][1] + eps);
                            if (!(ar > 2.0f && fr > 2.0f)) {
                                bb = uniq[ci];
                                bs = sc[ci][0];
                                bfn = sc[ci][1];
                                ban = sc[ci][2];
                            }
                            break;
                        }
                    }
                }
            }
            float conf = 0.0f;
            if (bs > 1e-12f) {
                const float ss = nu > 1 ? sc[keys[1] & 0xffffffffu][0] : 0.0f;
                conf = sd_clampf(sd_maxf(bs - ss, 0.0f) / bs, 0.0f, 1.0f);
            }
            int ag = 0;
            if (fft_pb > 0.0f && sd_absf(fft_pb - bb) < 2.0f) ag++;
            if (ac_pb > 0.0f && sd_absf(ac_pb - bb) < 2.0f) ag++;
            r.bpm = bb;
            r.conf = conf;
            r.agree = ag;
            r.ok = 1;
            const int nkeep = nu < P.top_n ? nu : P.top_n;
            r.n_cands = nkeep < cand_cap ? nkeep : cand_cap;
            float* co = cand + (uint64_t)item * cand_cap * 4;
            for (int k = 0; k < r.n_cands; k++) {
                const int ci = (int)(keys[k] & 0xffffffffu);
                co[4 * k + 0] = uniq[ci];
                co[4 * k + 1] = sc[ci][0];
                co[4 * k + 2] = sc[ci][1];
                co[4 * k + 3] = sc[ci][2];
            }
            if (P.gate) {  // src/lib.rs:412-459 on the candidates truncated to base_top_n
                const int ng = nu < P.gate_top_n ? nu : P.gate_top_n;
                auto support = [&](float q) {
                    float b = 0.0f;
                    for (int k = 0; k < ng; k++) {
                        const int ci = (int)(keys[k] & 0xffffffffu);
                        if (sd_absf(uniq[ci] - q) <= P.gate_tol) b = sd_maxf(b, sc[ci][0]);
                    }
                    return b;
                };
                const bool tl = bb >= 55.0f && bb <= 80.0f;
                const bool th = bb >= 170.0f && bb <= 200.0f;
                const float s_base = support(bb), s_2x = support(bb * 2.0f), s_half = support(bb * 0.5f);
                const bool fam = (s_2x > 0.0f && s_2x >= s_base * 0.90f) || (s_half > 0.0f && s_half >= s_base * 0.90f);
                const bool fold_into_trap = bb * 2.0f >= 170.0f && bb * 2.0f <= 200.0f;
                const bool weak = ag == 0 || conf < 0.06f;
                r.ambiguous = tl || th || fam || (weak && fold_into_trap);
                r.trap_low = tl;
                r.trap_high = th;
            }
            est[item] = r;
        }
    }
}

// ----------------------------------------------------------------------------------------
// Multi-resolution fusion (multi_resolution.rs:272-901) + acceptance (src/lib.rs:511-545).
// One 64-lane wave per track: lane 0 runs the decision logic; beat_contrast_score's phase
// loop is spread over the lanes (each phase's sums stay sequential; the max over phases is
// order-free).
constexpr int MR_CAP_LDS = 256;
// window maxima staged in LDS per segment of novelty frames (beat_contrast_seg): 16 KB whatever
// the track length, so a k_multires workgroup fits beside the key stream's STFT workgroups
constexpr int MR_SEG_BUF = 4096;
struct CandList {
    const float* c;  // 4 floats per candidate: bpm, score, fft_norm, ac_norm
    int n;
};

__device__ float lookup_c(CandList L, float bpm, float tol) {
    float bd = SD_INF_F, bs = 0.0f;
    for (int i = 0; i < L.n; i++) {
        const float d = sd_absf(L.c[4 * i] - bpm);
        if (d <= tol && d < bd) {
            bd = d;
            bs = L.c[4 * i + 1];
        }
    }
    return bs;
}

// beat_contrast_score (multi_resolution.rs:162-203) by the whole wave.  nov_total:
// novelty.iter().sum() (sequential), computed once per track by the caller.  Lane l owns the
// phases l + 64 q (q < 8; period <= 512).  The novelty's +-2 window maxima are staged in LDS one
// segment at a time (wbuf: MR_SEG_BUF floats; a segment of MR_SEG_BUF - period frames plus a halo
// of `period` frames, since the half- and third-beat lookups reach at most i + 2 period / 3), and
// each phase's sums visit their frames in increasing order across the segments: the same f32
// folds as one pass over the whole track.  The max over phases is order-free.
__device__ float beat_contrast_seg(const float* nov, int n, int sr, int hop, float bpm, float nov_total, float* wbuf) {
    if (n < 16 || !(sd_isfinite_f(bpm) && bpm > 0.0f) || sr == 0 || hop == 0) return 0.0f;
    const float fpb = (60.0f * (float)sr) / (bpm * (float)hop);
    if (!sd_isfinite_f(fpb) || fpb < 3.0f) return 0.0f;
    const int64_t pi = sd_f2i64(sd_roundf(fpb));
    if (!(pi >= 3 && pi <= 512)) return 0.0f;
    const int period = (int)pi, w = 2;
    const float total = sd_maxf(nov_total, 1e-6f);
    const int lane = threadIdx.x;  // blockDim == 64
    constexpr int NQ = 512 / 64;
    float bs[NQ], hs[NQ], ts[NQ];
    uint32_t bn[NQ], hn[NQ], tn[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) bs[q] = hs[q] = ts[q] = 0.0f, bn[q] = hn[q] = tn[q] = 0u;
    const int seg = MR_SEG_BUF - period;
    for (int s0 = 0; s0 < n; s0 += seg) {
        const int s1 = s0 + seg < n ? s0 + seg : n;
        const int e1 = s1 + period < n ? s1 + period : n;
        __syncthreads();  // the previous segment's reads are done
        for (int q = lane; q < e1 - s0; q += 64) {
            const int i = s0 + q;
            const int s = i >= w ? i - w : 0, e = i + w + 1 < n ? i + w + 1 : n;
            float mx = 0.0f;
            for (int j = s; j < e; j++) mx = sd_maxf(mx, nov[j]);
            wbuf[q] = mx;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int ph = lane + 64 * q;
            if (ph >= period) continue;
            int i = ph >= s0 ? ph : ph + ((s0 - ph + period - 1) / period) * period;
            for (; i < s1; i += period) {
                bs[q] += wbuf[i - s0];
                bn[q]++;
                if (period >= 6) {
                    const int j = i + period / 2;
                    if (j < n) {
                        hs[q] += wbuf[j - s0];
                        hn[q]++;
                    }
                }
                if (period >= 9) {
                    for (int fr = 1; fr <= 2; fr++) {
                        const int j = i + (period * fr) / 3;
                        if (j < n) {
                            ts[q] += wbuf[j - s0];
                            tn[q]++;
                        }
                    }
                }
            }
        }
    }
    float best = -1e9f;
#pragma unroll
    for (int q = 0; q < NQ; q++) {
        if (lane + 64 * q >= period) continue;
        const float bm = bn[q] > 0 ? bs[q] / (float)bn[q] : 0.0f;
        const float hm = hn[q] > 0 ? hs[q] / (float)hn[q] : 0.0f;
        const float tm = tn[q] > 0 ? ts[q] / (float)tn[q] : 0.0f;
        const float contrast = bm - 0.60f * hm - 0.40f * tm;
        const float score = sd_clampf(contrast / sd_maxf(total / (float)n, 1e-6f), -10.0f, 10.0f);
        best = sd_maxf(best, score);
    }
    return wave_max(best);
}

__global__ __launch_bounds__(64) void k_multires(const int* __restrict__ tracks, int n_items,
                                                 const float* __restrict__ c256, const int* __restrict__ n256,
                                                 const float* __restrict__ c512, const int* __restrict__ n512,
                                                 const float* __restrict__ c1024, const int* __restrict__ n1024,
                                                 int cap256, int cap512, int cap1024,
                                                 const TempoEst* __restrict__ base_est,
                                                 const float* __restrict__ nov512, const uint64_t* __restrict__ fpfx512,
                                                 MrParams P, TempoEst* __restrict__ mr_est, int* __restrict__ used,
                                                 float* __restrict__ final_bpm, float* __restrict__ final_conf,
                                                 MrDbg* __restrict__ dbg) {
    SDSP_LATENCY_CRITICAL();
    __shared__ float fam_bpm[5], fam_sup[5], fam_align[5];
    __shared__ int n_fam_s, do_fam_s;
    __shared__ int fam_lab[5];
    MrDbg dr{};  // thread 0's debug record (dbg only)
    __shared__ float best_bpm_s, best_score_s, second_s;
    __shared__ int ok_s;
    const int i = blockIdx.x;
    const int trk = tracks[i];
    const int j512 = P.own512 ? i : trk;  // index of this item's hop-512 data
    if (n256[i] < 0 || n1024[i] < 0 || n512[j512] < 0) {  // a hop's tempogram failed: multi_resolution returns Err
        if (threadIdx.x == 0) {
            mr_est[i].ok = 0;
            used[trk] = 0;
        }
        return;
    }
    // candidate lists staged in LDS when they fit (lane 0's lookups are latency-bound)
    __shared__ float s_c[3][4 * MR_CAP_LDS];
    CandList L256{c256 + (uint64_t)i * cap256 * 4, n256[i]};
    CandList L512{c512 + (uint64_t)j512 * cap512 * 4, n512[j512]};
    CandList L1024{c1024 + (uint64_t)i * cap1024 * 4, n1024[i]};
    CandList* Ls[3] = {&L256, &L512, &L1024};
    for (int l = 0; l < 3; l++) {
        CandList& L = *Ls[l];
        if (L.n <= MR_CAP_LDS) {
            for (int k = threadIdx.x; k < 4 * L.n; k += blockDim.x) s_c[l][k] = L.c[k];
            L.c = s_c[l];
        }
    }
    __syncthreads();
    const float tol = P.tol;
    if (threadIdx.x == 0) {
        ok_s = 0;
        struct Hyp {
            float bpm, score;
        };
        Hyp hyps[64];
        int nh = 0;
        const int kmax = P.top_k < L512.n ? P.top_k : L512.n;
        for (int ti = 0; ti < kmax && nh < 64; ti++) {
            const float t = L512.c[4 * ti];
            if (!(sd_isfinite_f(t) && t > 0.0f)) continue;
            const float st512 = lookup_c(L512, t, tol), st256 = lookup_c(L256, t, tol), st1024 = lookup_c(L1024, t, tol);
            const float s2512 = lookup_c(L512, t * 2.0f, tol), s2256 = lookup_c(L256, t * 2.0f, tol),
                        s21024 = lookup_c(L1024, t * 2.0f, tol);
            const float sh512 = lookup_c(L512, t * 0.5f, tol), sh256 = lookup_c(L256, t * 0.5f, tol),
                        sh1024 = lookup_c(L1024, t * 0.5f, tol);
            const float h_t = P.w512 * st512 + P.w256 * st256 + P.w1024 * st1024;
            float h_2t = P.w512 * (P.dt * st512 + (1.0f - P.dt) * s2512) + P.w256 * s2256 + P.w1024 * s21024;
            float h_h = P.w512 * (P.dt * st512 + (1.0f - P.dt) * sh512) + P.w256 * sh256 + P.w1024 * sh1024;
            if (st1024 > sh1024 * 1.02f) h_h *= 0.90f;
            if (st1024 > s21024 * 1.02f) h_2t *= 0.90f;
            const float eps = 1e-6f;
            const float r2 = (s2256 + eps) / (st256 + eps);
            if (r2 < 1.10f) h_2t *= 0.75f;
            if (r2 < 1.00f) h_2t *= 0.75f;
            const float rh = (sh1024 + eps) / (st1024 + eps);
            if (rh < 1.10f) h_h *= 0.75f;
            if (rh < 1.00f) h_h *= 0.75f;
            Hyp loc[3];
            int nl = 0;
            const Hyp cand3[3] = {{t, h_t}, {t * 2.0f, h_2t}, {t * 0.5f, h_h}};
            for (int k = 0; k < 3; k++)
                if (cand3[k].bpm >= P.min_bpm && cand3[k].bpm <= P.max_bpm) loc[nl++] = cand3[k];
            for (int k = 0; k < nl; k++) {
                if (loc[k].bpm > 210.0f)
                    loc[k].score *= 0.80f;
                else if (loc[k].bpm > 180.0f)
                    loc[k].score *= 0.90f;
                else if (loc[k].bpm < 60.0f)
                    loc[k].score *= 0.92f;
            }
            // stable sort desc (<= 3 entries)
            for (int a = 1; a < nl; a++) {
                Hyp tmp = loc[a];
                int b = a;
                while (b > 0 && loc[b - 1].score < tmp.score) {
                    loc[b] = loc[b - 1];
                    b--;
                }
                loc[b] = tmp;
            }
            if (nl == 0) continue;
            const float ss = nl > 1 ? loc[1].score : 0.0f;
            const float margin = loc[0].score - ss;
            float cb = loc[0].bpm, cs = loc[0].score;
            if (sd_absf(cb - t) > 1e-3f && margin < P.margin_thr) {
                cb = t;
                cs = h_t;
            }
            if (margin < P.margin_thr && P.human_prior && cb >= 70.0f && cb <= 180.0f && margin < 0.05f) cs += 0.05f;
            hyps[nh++] = {cb, cs};
        }
        if (nh > 0) {
            // stable sort desc by score
            for (int a = 1; a < nh; a++) {
                Hyp tmp = hyps[a];
                int b = a;
                while (b > 0 && hyps[b - 1].score < tmp.score) {
                    hyps[b] = hyps[b - 1];
                    b--;
                }
                hyps[b] = tmp;
            }
            Hyp uq[8];
            int nuq = 0;
            for (int a = 0; a < nh; a++) {
                bool dup = false;
                for (int b = 0; b < nuq; b++) dup |= sd_absf(uq[b].bpm - hyps[a].bpm) < 0.75f;
                if (dup) continue;
                uq[nuq++] = hyps[a];
                if (nuq >= 8) break;
            }
            Hyp best = uq[0];
            auto total_support = [&](float bpm, float* s, int* a) {
                const float x1 = lookup_c(L256, bpm, tol), x2 = lookup_c(L512, bpm, tol), x3 = lookup_c(L1024, bpm, tol);
                *a = (x1 > 0.0f) + (x2 > 0.0f) + (x3 > 0.0f);
                *s = x1 + x2 + x3;
            };
            if (best.bpm >= 170.0f) {
                const float half = best.bpm * 0.5f;
                if (half >= 70.0f && half <= 120.0f) {
                    float sb, sh;
                    int ab, ah;
                    total_support(best.bpm, &sb, &ab);
                    total_support(half, &sh, &ah);
                    const float ratio = sb > 0.0f ? sh / sb : 0.0f;
                    if (ah >= 3 && sh > 0.0f && sb > 0.0f && ratio >= 0.45f) {
                        dr.fd = 1, dr.fd_from = best.bpm, dr.fd_to = half, dr.fd_ratio = ratio, dr.fd_a0 = ab, dr.fd_a1 = ah;
                        best = {half, sh};
                    }
                }
            }
            if (best.bpm <= 80.0f) {
                const float dbl = best.bpm * 2.0f;
                if (dbl >= 70.0f && dbl <= 180.0f) {
                    float sb, sd;
                    int ab, ad;
                    total_support(best.bpm, &sb, &ab);
                    total_support(dbl, &sd, &ad);
                    const float ratio = sb > 0.0f ? sd / sb : 0.0f;
                    if (ad >= 2 && sd > 0.0f && sb > 0.0f && ratio >= 0.55f) {
                        dr.fu = 1, dr.fu_from = best.bpm, dr.fu_to = dbl, dr.fu_ratio = ratio, dr.fu_a0 = ab, dr.fu_a1 = ad;
                        best = {dbl, sd};
                    }
                }
            }
            // triplet-family candidates (alignment computed by the whole wave below)
            int nf = 0;
            if (P.band && best.bpm >= 70.0f && best.bpm <= 180.0f) {
                const float ff[5] = {1.0f, 3.0f / 2.0f, 2.0f / 3.0f, 4.0f / 3.0f, 3.0f / 4.0f};
                for (int k = 0; k < 5; k++) {
                    const float bpm = best.bpm * ff[k];
                    if (!(sd_isfinite_f(bpm) && bpm >= P.min_bpm && bpm <= P.max_bpm)) continue;
                    if (!(bpm >= 70.0f && bpm <= 180.0f)) continue;
                    float sup;
                    int ag;
                    total_support(bpm, &sup, &ag);
                    if (ag < 2 || sup <= 0.0f) continue;
                    fam_bpm[nf] = bpm;
                    fam_sup[nf] = sup;
                    fam_lab[nf] = k;
                    nf++;
                }
            }
            n_fam_s = nf;
            best_bpm_s = best.bpm;
            best_score_s = best.score;
            second_s = nuq > 1 ? uq[1].score : 0.0f;
            ok_s = 1;
        }
    }
    __syncthreads();
    if (!ok_s) {
        if (threadIdx.x == 0) {
            mr_est[i].ok = 0;
            used[trk] = 0;
        }
        return;
    }
    const int nf = n_fam_s;
    const uint64_t g0 = fpfx512[j512];
    const int nn = (int)(fpfx512[j512 + 1] - g0) - 1;
    const float* nov = nov512 + g0;
    // one LDS buffer: block_seq_sum's staging (SEQ_CH), then beat_contrast_seg's segments
    __shared__ float wbuf[MR_SEG_BUF];
    static_assert(MR_SEG_BUF >= SEQ_CH, "the staging buffer is shared");
    const float nov_total = (nf >= 2 && nn > 0) ? block_seq_sum(nov, nn, wbuf) : 0.0f;
    if (nf >= 2 && nn > 0) {
        for (int k = 0; k < nf; k++) {
            const float a = beat_contrast_seg(nov, nn, P.sr, P.hop512, fam_bpm[k], nov_total, wbuf);
            if (threadIdx.x == 0) fam_align[k] = a;
            __syncthreads();
        }
    }
    float cur_align = 0.0f;
    if (threadIdx.x == 0 && nf >= 2 && nn > 0) {
        float bs = 0.0f;
        for (int k = 0; k < nf; k++) bs = sd_maxf(bs, fam_sup[k]);
        bs = sd_maxf(bs, 1e-6f);
        float max_alt = 0.0f;
        for (int k = 0; k < nf; k++)
            if (sd_absf(fam_bpm[k] - best_bpm_s) > 0.75f) max_alt = sd_maxf(max_alt, fam_sup[k] / bs);
        do_fam_s = max_alt >= 0.45f;
        if (do_fam_s) {
            int ch = 0;
            float cs = -1e9f;
            for (int k = 0; k < nf; k++) {
                const float sn = sd_clampf(fam_sup[k] / bs, 0.0f, 1.0f);
                const float s = fam_align[k] + 0.35f * sn;
                if (s > cs) {
                    ch = k;
                    cs = s;
                }
            }
            fam_bpm[0 + 4] = fam_bpm[ch];  // stash chosen
            fam_sup[0 + 4] = fam_sup[ch];
            fam_align[4] = fam_align[ch];
            if (dbg) {  // current.support (total_support of the best) and the chosen's, over the best family support
                const float sc = lookup_c(L256, best_bpm_s, tol) + lookup_c(L512, best_bpm_s, tol) +
                                 lookup_c(L1024, best_bpm_s, tol);
                dr.tf_sup0 = sc / bs;
                dr.tf_sup1 = fam_sup[ch] / bs;
                dr.tf_label = fam_lab[ch];
            }
        }
    } else if (threadIdx.x == 0) {
        do_fam_s = 0;
    }
    __syncthreads();
    if (do_fam_s) {
        cur_align = beat_contrast_seg(nov, nn, P.sr, P.hop512, best_bpm_s, nov_total, wbuf);
        if (threadIdx.x == 0) {
            if (sd_absf(fam_bpm[4] - best_bpm_s) > 0.75f && fam_align[4] >= cur_align + 0.40f) {
                dr.tf = 1, dr.tf_from = best_bpm_s, dr.tf_to = fam_bpm[4], dr.tf_al0 = cur_align, dr.tf_al1 = fam_align[4];
                best_bpm_s = fam_bpm[4];
                best_score_s = fam_sup[4];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float bb = best_bpm_s, bsc = best_score_s;
        const float conf = bsc > 1e-6f ? sd_clampf(sd_maxf(bsc - second_s, 0.0f) / bsc, 0.0f, 1.0f) : 0.0f;
        const int agree = (lookup_c(L256, bb, tol) > 0.0f) + (lookup_c(L512, bb, tol) > 0.0f) +
                          (lookup_c(L1024, bb, tol) > 0.0f);
        TempoEst m{};
        m.bpm = bb;
        m.conf = conf;
        m.agree = agree;
        m.ok = 1;
        mr_est[i] = m;
        // acceptance (src/lib.rs:515-545)
        const TempoEst b = base_est[trk];
        const float rel = b.bpm > 1e-6f ? sd_maxf(bb / b.bpm, b.bpm / bb) : 1.0f;
        const bool fam = sd_absf(rel - 2.0f) < 0.05f || sd_absf(rel - 1.5f) < 0.05f || sd_absf(rel - (4.0f / 3.0f)) < 0.05f;
        const bool forbid = b.bpm <= 180.0f && bb > 180.0f;
        const bool better = !forbid && (conf >= (b.conf + 0.05f) || (agree > b.agree && conf >= b.conf * 0.90f) ||
                                        ((b.trap_low || b.trap_high) && fam && conf >= b.conf * 0.88f &&
                                         ((bb >= 70.0f && bb <= 180.0f) || b.bpm > 180.0f)));
        used[trk] = better;
        if (better) {
            final_bpm[trk] = bb;
            final_conf[trk] = conf;
        }
        if (dbg) {
            dr.rel = rel, dr.fam = fam, dr.forbid = forbid, dr.better = better;
            dbg[i] = dr;
        }
    }
}

// ---- launchers ----
void launch_fft_tempogram(const int* items, int n_items, int T, const float* nov, const float* nov_sum,
                          const uint64_t* frame_pfx, uint64_t total, const FftTgParams& P, const cx* tw, const cx* rt,
                          cx* gscratch, const uint64_t* out_off, float* out_bpm, float* out_pow, hipStream_t st) {
    if (n_items == 0) return;
    int K2 = 1;
    while (K2 < P.K) K2 <<= 1;
    const size_t lds = P.lds ? (size_t)(P.P / 2 + K2) * sizeof(cx) : 0;  // M = P/2 slots + keys
    if (P.lds)
        hipLaunchKernelGGL(k_fft_tempogram<true>, dim3(n_items), dim3(256), lds, st, items, n_items, T, nov, nov_sum,
                           frame_pfx, total, P, tw, rt, gscratch, out_off, out_bpm, out_pow);
    else
        hipLaunchKernelGGL(k_fft_tempogram<false>, dim3(n_items), dim3(256), 0, st, items, n_items, T, nov, nov_sum,
                           frame_pfx, total, P, tw, rt, gscratch, out_off, out_bpm, out_pow);
}
void launch_acf_tempogram(const int* items, int n_items, const float* nov, const uint64_t* frame_pfx, uint64_t total,
                          const float* bpm_grid, const int* lag_grid, int NB, float* out_bpm, float* out_str,
                          hipStream_t st) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_acf_tempogram, dim3(n_items), dim3(256), 0, st, items, nov, frame_pfx, total, bpm_grid,
                       lag_grid, NB, out_bpm, out_str);
}
void launch_tempo_select(int n_items, const int* active, const float* fft_bpm, const float* fft_pow, const uint64_t* fft_off,
                         const int* fft_k, const float* acf_bpm, const float* acf_str, const uint64_t* acf_off,
                         const SelParams& P, TempoEst* est, float* cand, int cand_cap, hipStream_t st) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_tempo_select, dim3(n_items), dim3(256), 0, st, active, n_items, fft_bpm, fft_pow,
                       fft_off, fft_k, acf_bpm, acf_str, acf_off, P, est, cand, cand_cap);
}
void launch_multires(const int* tracks, int n_items, const float* c256, const int* n256, const float* c512,
                     const int* n512, const float* c1024, const int* n1024, int cap256, int cap512, int cap1024,
                     const TempoEst* base_est, const float* nov512, const uint64_t* fpfx512, const MrParams& P,
                     TempoEst* mr_est, int* used, float* final_bpm, float* final_conf, hipStream_t st, MrDbg* dbg) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_multires, dim3(n_items), dim3(64), 0, st, tracks, n_items, c256, n256, c512, n512, c1024,
                       n1024, cap256, cap512, cap1024, base_est, nov512, fpfx512, P, mr_est, used, final_bpm,
                       final_conf, dbg);
}

}  // namespace sdsp
