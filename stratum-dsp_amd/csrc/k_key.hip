// k_key.hip — key detection path (reference src/lib.rs:961-1559):
//
//   k_mask      harmonic_spectrogram_time_mask + smooth_spectrogram_time  chroma/extractor.rs:1246-1349
//   k_hpcp      HPCP chroma + frame energies                              extractor.rs:529-680, 1097-1150
//   k_key_vote  median smoothing, frame weights, segment voting,         smoothing.rs:37-94, src/lib.rs:1211-1436,
//               detect_key_weighted, key clarity                          key/detector.rs:68-313, key_clarity.rs:51-93
//
// k_mask: one thread per (track, bin) streams the track's frames in order, carrying the
// reference's sequential per-bin f32 prefix sum (prefix[t+1] = prefix[t] + x) in a 2M+2-slot
// ring in LDS; adjacent lanes touch adjacent bins of the same frame, so every HBM access is a
// coalesced 1 KB row segment.  The mask is applied in place.
#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdsp {

constexpr int MASK_T = 64;  // bins per workgroup (one wave): 4097 bins = 64 full waves + 1 lane
constexpr int MASK_U = 16;  // frames loaded ahead per thread (independent HBM loads in flight)

// LDS: prefix ring pre[2M+2][MASK_T] and raw ring raw[M+1][MASK_T] (dynamic, sized by M).
// Ring slots advance by counters (no runtime modulo): the prefix for en = min(t+M+1, F) is
// always the last one written; st = max(t-M, 0) advances once t > M; raw[t] was written M
// frames earlier.
// PW: 2 -> power 2 (x*x, the default), 1 -> power 1, 0 -> any other power (sd_powf); keeps the
// unrolled body free of the general pow code.
template <int PW>
__device__ __forceinline__ float mask_pow(float x, float p) {
    if (PW == 2) return x * x;
    if (PW == 1) return x;
    return sd_powf(x, p);
}

template <int PW>
__global__ __launch_bounds__(MASK_T) void k_mask(float* __restrict__ mags, int stride, int B,
                                                  const uint64_t* __restrict__ frame_pfx, const int* __restrict__ tracks,
                                                  int blocks_per_track, int margin, float power, int smooth_only) {
    extern __shared__ float mask_lds[];
    const int it = blockIdx.x / blocks_per_track;
    const int trk = tracks[it];
    const int b = (blockIdx.x % blocks_per_track) * MASK_T + threadIdx.x;
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    if (b >= B || F <= 0) return;
    float* col = mags + frame_pfx[trk] * (uint64_t)stride + b;
    const int M = margin;
    const int R = 2 * M + 2, RX = M + 1;
    float* pre = mask_lds + threadIdx.x;
    float* raw = mask_lds + (size_t)R * MASK_T + threadIdx.x;
    const float p = sd_maxf(power, 1.0f);
    const float eps = 1e-12f;
    pre[0] = 0.0f;
    float prev = 0.0f;
    int w_slot = 0;   // slot of prefix[min(tin+1, F)] after this step's write (= en's slot)
    int s_slot = 0;   // slot of prefix[st]
    int xw = 0;       // raw write slot (tin % RX)
    int xr = 0;       // raw read slot (t % RX)
    for (int64_t base = 0; base < F + M; base += MASK_U) {
        float xv[MASK_U];
#pragma unroll
        for (int u = 0; u < MASK_U; u++) {
            const int64_t tin = base + u;
            xv[u] = tin < F ? col[tin * stride] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < MASK_U; u++) {
            const int64_t tin = base + u;
            if (tin >= F + M) break;
            if (tin < F) {
                prev = prev + xv[u];
                w_slot = w_slot + 1 == R ? 0 : w_slot + 1;
                pre[w_slot * MASK_T] = prev;
                raw[xw * MASK_T] = xv[u];
                xw = xw + 1 == RX ? 0 : xw + 1;
            }
            const int64_t t = tin - M;
            if (t < 0) continue;
            const int64_t st = t >= M ? t - M : 0;
            const int64_t en = t + M + 1 < F ? t + M + 1 : F;
            const float denom = (float)(en - st > 1 ? en - st : 1);
            const float x_raw = M == 0 ? xv[u] : raw[xr * MASK_T];
            // margin 0: smooth_spectrogram_time returns its input unchanged (extractor.rs:1250-1252)
            const float hm = M == 0 ? x_raw : (pre[w_slot * MASK_T] - pre[s_slot * MASK_T]) / denom;
            if (smooth_only) {  // smooth_spectrogram_time alone (src/lib.rs:1042-1055)
                col[t * stride] = hm;
                if (M > 0) xr = xr + 1 == RX ? 0 : xr + 1;
                if (t >= M) s_slot = s_slot + 1 == R ? 0 : s_slot + 1;
                continue;
            }
            const float x = max_bnn(x_raw, 0.0f);
            const float h = max_bnn(hm, 0.0f);
            const float r = max_bnn(x - h, 0.0f);
            const float hp = mask_pow<PW>(h, p);
            const float rp = mask_pow<PW>(r, p);
            const float m = hp / (hp + rp + eps);
            col[t * stride] = x * m;
            if (M > 0) xr = xr + 1 == RX ? 0 : xr + 1;
            if (t >= M) s_slot = s_slot + 1 == R ? 0 : s_slot + 1;
        }
    }
}

// Register-ring variant for a compile-time margin M (the default 12): the prefix ring
// (R = 2M+2 slots) and the raw ring (M+1 slots) live in VGPRs and the frame loop is unrolled
// by R, so every slot index is static.  Edges need no special case: frames past the end
// contribute x = 0 (prefix + 0 == prefix, so P[min(t+M+1, F)] is read as P[t+M+1]), and
// prefixes of negative index are the ring's initial zeros (== P[0]) because slot (t-M) mod R
// is not written before t >= M.  R loads are issued ahead of each unrolled block.
// One masked element: window sum a over `den` frames and the raw value xr -> xr * mask
// (extractor.rs:1281-1285 then 1320-1340).  For the full window (2M+1 frames) a/(2M+1) is one
// product and one FMA correction, == the correctly rounded quotient for every f32 a in
// {0} U [2^-90, 2^120] (tools/check_div.c: exhaustive, every odd window 3..25); otherwise the
// IEEE division.
template <int M, int PW>
__device__ __forceinline__ float mask_elem(float a, int64_t den, float xr, float p, float inv_w) {
    float hm;
    if (den == 2 * M + 1 && (a == 0.0f || (a >= 0x1p-90f && a <= 0x1p120f))) {
        const float q0 = a * inv_w;
        hm = __builtin_fmaf(__builtin_fmaf(-q0, (float)(2 * M + 1), a), inv_w, q0);
    } else {
        hm = a / (float)(den > 1 ? den : 1);
    }
    const float x = max_bnn(xr, 0.0f);
    const float h = max_bnn(hm, 0.0f);
    const float r = max_bnn(x - h, 0.0f);
    const float hp = mask_pow<PW>(h, p);
    const float rp = mask_pow<PW>(r, p);
    const float m = hp / (hp + rp + 1e-12f);
    return x * m;
}

template <int M, int PW>
__global__ __launch_bounds__(MASK_T) void k_mask_r(float* __restrict__ mags, int stride, int B,
                                                    const uint64_t* __restrict__ frame_pfx,
                                                    const int* __restrict__ tracks, int blocks_per_track,
                                                    float power) {
    constexpr int R = 2 * M + 2, RX = M + 1;
    static_assert(M >= 1 && (2 * M + 1) % 2 == 1 && 2 * M + 1 <= 25, "fast window division validated for 3..25");
    const int it = blockIdx.x / blocks_per_track;
    const int trk = tracks[it];
    const int b = (blockIdx.x % blocks_per_track) * MASK_T + threadIdx.x;
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    if (b >= B || F <= 0) return;
    float* col = mags + frame_pfx[trk] * (uint64_t)stride + b;
    const float p = sd_maxf(power, 1.0f);
    const float inv_w = 1.0f / (float)(2 * M + 1);
    float P[R], X[RX];
#pragma unroll
    for (int j = 0; j < R; j++) P[j] = 0.0f;
#pragma unroll
    for (int j = 0; j < RX; j++) X[j] = 0.0f;
    float prev = 0.0f;
    auto emit = [&](float a, int64_t den, float xr, int64_t t) {
        __builtin_nontemporal_store(mask_elem<M, PW>(a, den, xr, p, inv_w), &col[t * stride]);
    };
    for (int64_t base = 0; base < F + M; base += R) {
        float xv[R];
        if (base >= 2 * M && base + R <= F) {
            // interior block: every step has a full window; no edge conditions
#pragma unroll
            for (int u = 0; u < R; u++) xv[u] = __builtin_nontemporal_load(&col[(base + u) * stride]);
#pragma unroll
            for (int u = 0; u < R; u++) {
                prev = prev + xv[u];
                P[(u + 1) % R] = prev;
                X[u % RX] = xv[u];
                emit(P[(u + 1) % R] - P[(u + R - 2 * M) % R], 2 * M + 1, X[(u + 1) % RX], base + u - M);
            }
            continue;
        }
#pragma unroll
        for (int u = 0; u < R; u++) xv[u] = base + u < F ? __builtin_nontemporal_load(&col[(base + u) * stride]) : 0.0f;
#pragma unroll
        for (int u = 0; u < R; u++) {
            const int64_t tin = base + u;
            prev = prev + xv[u];  // == prev once tin >= F (x = 0)
            P[(u + 1) % R] = prev;
            X[u % RX] = xv[u];
            const int64_t t = tin - M;
            if (t >= 0 && t < F) {
                const int64_t st = t >= M ? t - M : 0;
                const int64_t en = t + M + 1 < F ? t + M + 1 : F;
                emit(P[(u + 1) % R] - P[(u + R - 2 * M) % R], en - st, X[(u + 1) % RX], t);
            }
        }
    }
}

// k_mask_rp: k_mask_r for the default HPCP path, which reads the masked spectrogram only on its
// peak band [st_lo, st_hi] (extractor.rs:583-671: peaks in [pk_lo, pk_hi] and their neighbours)
// and otherwise only folds the frame energy sum(x * x) over every bin (extractor.rs:1133).  The
// masked value is stored only on that band; for every frame the workgroup's 64 bins (block g) fold
// their squares into part[g][frame] (an LDS tile: lane = bin writes, then lanes u and u + 32 fold the
// two 32-bin halves of the row of frame base + u - M in bin order and the halves are added), and
// HPCP folds the 65 block sums in block order.  Only that fold's association differs from the
// reference's one sequential sum over 4,097 bins (a GPU-only re-association of the key energies,
// DESIGN.md §2); every masked value is bit-identical.
// Lanes past the last bin stay in the wave and contribute +0 (exact: the sums are >= +0).
// the block fold's chains: 1 = lane u folds the 64 squares of frame u alone; 2 (default) = lanes u
// and u + 32 fold 32 each and add the halves (-1.8 % per launch, profiles/r06_kernel_ab_mask_fold.txt;
// 4 = two interleaved chains of 16 per lane, -0.8 %)
#ifndef SDSP_MASK_FOLD_CH
#define SDSP_MASK_FOLD_CH 2
#endif
template <int M, int PW>
__global__ __launch_bounds__(MASK_T) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_mask_rp(float* __restrict__ mags, int stride, int B,
                                                     const uint64_t* __restrict__ frame_pfx,
                                                     const int* __restrict__ tracks, int blocks_per_track,
                                                     float power, int st_lo, int st_hi, float* __restrict__ part,
                                                     uint64_t total, int outside) {
    constexpr int R = 2 * M + 2, RX = M + 1;
    static_assert(M >= 1 && 2 * M + 1 <= 25 && R <= MASK_T, "fast window division validated for 3..25");
    __shared__ float tile[R][MASK_T + 1];
    const int it = blockIdx.x / blocks_per_track;
    const int trk = tracks[it];
    const int gblk = blockIdx.x % blocks_per_track;
    const int lane = threadIdx.x;
    const int b = gblk * MASK_T + lane;
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    if (F <= 0) return;  // the whole workgroup
    // outside: store the bins outside [st_lo, st_hi] instead (the exact rerun's completion of a
    // spectrogram whose band already holds masked values); a block wholly inside stores nothing
    if (outside && gblk * MASK_T >= st_lo && gblk * MASK_T + MASK_T - 1 <= st_hi) return;
    const bool live = b < B;
    const bool keep = live && (outside ? (b < st_lo || b > st_hi) : (b >= st_lo && b <= st_hi));
    // Rows are addressed through buffer resources whose base is the row (wave-uniform, advanced in
    // SGPRs) and lane offsets in VGPRs: no 64-bit address arithmetic per element.  A store
    // resource spans one row (B floats) and the lanes off HPCP's band carry an offset past it, so
    // the hardware drops their stores without an exec-mask branch per element.
    float* const trk0 = mags + frame_pfx[trk] * (uint64_t)stride;
    const uint32_t lvo = (uint32_t)(live ? b : 0) * 4u;
    // lanes past the last bin load through an offset past the row resource's range: the hardware
    // returns 0 without an exec-mask branch per load
    const uint32_t lvo_z = live ? (uint32_t)b * 4u : 0x80000000u;
    const uint32_t svo = keep ? (uint32_t)b * 4u : 0x80000000u;
    const uint32_t rowb = (uint32_t)stride * 4u;
    auto row_rsrc = [&](int64_t row, uint32_t bytes) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(trk0 + row * (int64_t)stride), (short)0, (int)bytes, 0x00020000);
    };
    float* pg = part + (uint64_t)gblk * total + frame_pfx[trk];
    const float p = sd_maxf(power, 1.0f);
    const float inv_w = 1.0f / (float)(2 * M + 1);
    float P[R], X[RX];
#pragma unroll
    for (int j = 0; j < R; j++) P[j] = 0.0f;
#pragma unroll
    for (int j = 0; j < RX; j++) X[j] = 0.0f;
    float prev = 0.0f;
    auto finish = [&](float v, int64_t t, int u) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), row_rsrc(t, (uint32_t)B * 4u), svo, 0, 2 /* nt */);
        tile[u][lane] = v * v;  // lanes past the last bin load x = 0, so v = 0 * (0 / 1e-12) = +0
    };
    // interior element: the full window's quotient by the product + FMA correction, exact on
    // {0} U [2^-90, 2^120] (mask_elem); a wave with a lane outside that range (tiny non-zero or huge
    // window sums) redoes that lane by the IEEE division, behind a wave-uniform branch.  chk =
    // false: the block's range test (below) already holds for every lane of the wave
    auto emit_full = [&](float a, float xr, int64_t t, int u, bool chk = true) {
        const float q0 = a * inv_w;
        float hm = __builtin_fmaf(__builtin_fmaf(-q0, (float)(2 * M + 1), a), inv_w, q0);
        // outside {+-0} U [2^-90, 2^120] (negative, NaN: sign or exponent bits above the range)
        const uint32_t ab = __float_as_uint(a);
        const bool bad = ((ab << 1) != 0u) & (ab - 0x12800000u > 0x7B800000u - 0x12800000u);
        if (chk && __builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0))
            if (bad) hm = a / (float)(2 * M + 1);
        // the block test (chk = false) also certifies every sample of the block and the ring finite
        // and >= +0, and then a >= +0 and its correctly rounded quotient hm >= +0: both max(., 0)
        // are the identity there
        const float x = chk ? max0_quiet(xr) : xr;
        const float h = chk ? max0_quiet(hm) : hm;
        const float r = max_bnn(x - h, 0.0f);
        const float hp = mask_pow<PW>(h, p);
        const float rp = mask_pow<PW>(r, p);
        const float den = hp + rp + 1e-12f;
        if (!chk) {  // the block's range test holds (below)
            const float y = __builtin_amdgcn_rcpf(den);
            const float y1 = __builtin_fmaf(__builtin_fmaf(-den, y, 1.0f), y, y);
            const float q0 = hp * y1;
            finish(x * __builtin_fmaf(__builtin_fmaf(-den, q0, hp), y1, q0), t, u);
            return;
        }
        finish(x * (hp / den), t, u);
    };
    // the block's partial sums: lane u folds the 64 squares of frame base + u - M in bin order
    auto fold = [&](int64_t base) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if SDSP_MASK_FOLD_CH == 1
        const int64_t t = base + lane - M;
        if (lane < R && t >= 0 && t < F) {
            float sum = 0.0f;
#pragma unroll 16
            for (int j = 0; j < MASK_T; j++) sum += tile[lane][j];
            pg[t] = sum;
        }
#else
        {
            // two lanes per frame (u, u + 32), each folding half of the block's bins in bin order
            // (SDSP_MASK_FOLD_CH / 2 interleaved chains each), the halves added at the end
            constexpr int NCH = SDSP_MASK_FOLD_CH / 2, CL = MASK_T / 2 / NCH;
            const int fu = lane & 31, hf = lane >> 5;
            const int64_t t = base + fu - M;
            float sc[NCH];
#pragma unroll
            for (int c = 0; c < NCH; c++) sc[c] = 0.0f;
            if (fu < R) {
#pragma unroll
                for (int j = 0; j < CL; j++)
#pragma unroll
                    for (int c = 0; c < NCH; c++) sc[c] += tile[fu][hf * (MASK_T / 2) + c * CL + j];
            }
            float sum = sc[0];
#pragma unroll
            for (int c = 1; c < NCH; c++) sum += sc[c];
            const float hi = __shfl_down(sum, 32);
            if (hf == 0 && fu < R && t >= 0 && t < F) pg[t] = sum + hi;
        }
#endif
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // the next block's loads are issued as soon as the current block's values are consumed, so
    // they are in flight during the block-sum fold (its 64-step chains would otherwise stall them)
    float xv[R];
    auto load_block = [&](int64_t base) {
        const auto rs = row_rsrc(base, 0x7FFFFFFFu);
        if (base >= 2 * M && base + R <= F) {
#pragma unroll
            for (int u = 0; u < R; u++) xv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lvo_z, (uint32_t)u * rowb, 2));
        } else {
#pragma unroll
            for (int u = 0; u < R; u++)
                xv[u] = (live && base + u < F) ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lvo, (uint32_t)u * rowb, 2))
                                               : 0.0f;
        }
    };
    load_block(0);
    for (int64_t base = 0; base < F + M; base += R) {
        if (base >= 2 * M && base + R <= F) {
            // interior block: every step has a full window; no edge conditions
            // the per-element range checks once per block.  P is non-decreasing and every window
            // sum a = P1 - P0 has P1 in [P[base + 1], P[base + R]]; a nonzero difference is at
            // least half an ulp of P1 (or P1 / 2), so a = 0 or a >= P[base + 1] 2^-25, and the
            // sequential prefix rounds up by at most (1 + 2^-24)^R, so a <= 2^60.01 when prev +
            // R max(x) <= 2^60.  With P[base + 1] >= 2^-21: a is 0 or in [2^-46, 2^61] (the window
            // quotient's exact range), hp = h^2 is 0 or >= 2^-103 (the mask quotient's residual is
            // exact), and with P[base + 1] >= max(x) 2^-31, hp / den >= 2^-124 (r <= x), hp, rp and
            // den stay below 2^112: the reciprocal + Newton + FMA-residual quotient is then the
            // correctly rounded one (tools/check_div_fast.hip, D1, every mantissa pair).  max(x)
            // covers the block's samples and the raw ring (the centres x of the block's first
            // elements are the previous block's).  A block and past of zeros is exact on either
            // path.  NaN and inf fail the tests.
            // max(x) over the block and the ring as unsigned bit patterns: for values with a clear
            // sign bit that is the float maximum, and a NaN, an infinity or a negative value (sign bit)
            // makes it >= 0x7F800000, so the test below also certifies every value finite and >= +0
            uint32_t mb = __float_as_uint(xv[0]);
#pragma unroll
            for (int u = 1; u < R; u++) mb = max(mb, __float_as_uint(xv[u]));
#pragma unroll
            for (int j = 0; j < RX; j++) mb = max(mb, __float_as_uint(X[j]));
            const float mx = __uint_as_float(mb);
            const float pf = prev + xv[0];
            const bool ok = mb < 0x7F800000u && (prev + mx == 0.0f || (pf >= 0x1p-21f && pf >= mx * 0x1p-31f &&
                                                                        prev + (float)R * mx <= 0x1p60f));
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) == 0, 1)) {
#pragma unroll
                for (int u = 0; u < R; u++) {
                    prev = prev + xv[u];
                    P[(u + 1) % R] = prev;
                    X[u % RX] = xv[u];
                    emit_full(P[(u + 1) % R] - P[(u + R - 2 * M) % R], X[(u + 1) % RX], base + u - M, u, false);
                }
            } else
#pragma unroll
            for (int u = 0; u < R; u++) {
                prev = prev + xv[u];
                P[(u + 1) % R] = prev;
                X[u % RX] = xv[u];
                emit_full(P[(u + 1) % R] - P[(u + R - 2 * M) % R], X[(u + 1) % RX], base + u - M, u);
            }
        } else {
#pragma unroll
            for (int u = 0; u < R; u++) {
                const int64_t tin = base + u;
                prev = prev + xv[u];  // == prev once tin >= F (x = 0)
                P[(u + 1) % R] = prev;
                X[u % RX] = xv[u];
                const int64_t t = tin - M;
                if (t >= 0 && t < F) {
                    const int64_t st = t >= M ? t - M : 0;
                    const int64_t en = t + M + 1 < F ? t + M + 1 : F;
                    finish(mask_elem<M, PW>(P[(u + 1) % R] - P[(u + R - 2 * M) % R], en - st, X[(u + 1) % RX], p, inv_w),
                           t, u);
                }
            }
        }
        if (base + R < F + M) load_block(base + R);
        fold(base);
    }
}

// ----------------------------------------------------------------------------------------
constexpr int HP_CW = 16;  // bins per staged chunk (LDS row stride 17: conflict-free)
constexpr int HPB_CW = HP_CW;  // k_hpcp_band's chunk (32: 164 VGPRs, 3 waves, 15 % slower in round 5)
static_assert(HPB_CW == 16, "k_hpcp_band stages a chunk as four 16-byte groups per row");

// The per-frame HPCP state of one thread (extractor.rs:529-680 for one frame): the energy fold,
// the last two magnitudes for the local-maximum test, and a register-resident top-KCAP list
// ordered (magnitude desc, bin asc).  KCAP is the compile-time list capacity (>= K); the
// insertion is branch-free straight-line code over the KCAP slots.  Slots K..KCAP-1 hold the
// runners-up and are ignored at the end (the first K slots are exactly the top-K in order).
// thr = pm[KCAP-1]: a candidate must beat it to move anything.
template <int KCAP>
struct HpcpFrame {
    float e = 0.0f, m1 = 0.0f, m2 = 0.0f;  // m1 = m[b-1], m2 = m[b-2]
    float thr = -1.0f;
    float pm[KCAP];
    int pb[KCAP];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int q = 0; q < KCAP; q++) {
            pm[q] = -1.0f;  // empty slot; every real peak is > 0
            pb[q] = 0;
        }
    }
    // bins c0 .. c0+cw-1 of this frame, row[j] = m[c0 + j], in bin order
    template <bool ENERGY = true>
    __device__ __forceinline__ void walk(const float* row, int c0, int cw, const HpcpParams& P) {
        for (int j = 0; j < cw; j++) {
            const int b = c0 + j;
            const float m = row[j];
            if (ENERGY) e += m * m;
            const int c = b - 1;  // candidate peak bin, needs m[c-1] = m2, m[c] = m1, m[c+1] = m
            if (c >= P.pk_lo && c <= P.pk_hi && !(m1 <= m2 || m1 < m) && m1 > thr) {
                // insertion into the descending list: gt[q] = m1 > pm[q] is false then true along
                // the list (an equal magnitude already listed has the lower bin and stays
                // ahead), so slot q takes m1 where gt turns true and its predecessor after that.
                // Updated from the tail in place: one compare and four selects per slot.
                bool gt[KCAP];
#pragma unroll
                for (int q = 0; q < KCAP; q++) gt[q] = m1 > pm[q];
#ifndef SDSP_HPCP_SELECT_PM
                // the magnitudes: slot q takes the median of {pm[q], m1, pm[q-1]} (pm[q-1] >= pm[q]:
                // that is pm[q] if m1 <= pm[q], m1 between the two, pm[q-1] if m1 > pm[q-1]), one
                // v_med3 instead of two selects; exact, every operand is a number (m1 > thr >= -1)
#pragma unroll
                for (int q = KCAP - 1; q >= 1; q--) {
                    const int nbv = gt[q - 1] ? pb[q - 1] : c;
                    pm[q] = __builtin_amdgcn_fmed3f(pm[q], m1, pm[q - 1]);
                    pb[q] = gt[q] ? nbv : pb[q];
                }
#else
#pragma unroll
                for (int q = KCAP - 1; q >= 1; q--) {
                    const float nv = gt[q - 1] ? pm[q - 1] : m1;
                    const int nbv = gt[q - 1] ? pb[q - 1] : c;
                    pm[q] = gt[q] ? nv : pm[q];
                    pb[q] = gt[q] ? nbv : pb[q];
                }
#endif
                pm[0] = gt[0] ? m1 : pm[0];
                pb[0] = gt[0] ? c : pb[0];
                thr = pm[KCAP - 1];
            }
            m2 = m1;
            m1 = m;
        }
    }
    // harmonic summation of the top-K peaks into 12 pitch classes (pc[q][i]: this thread's
    // column of an LDS scratch), L2 normalisation, and the frame's chroma row and energy at g
    template <int HU = 4>
    __device__ __forceinline__ void finish(float (*pc)[HP_FRAMES], int i, const HpcpParams& P,
                                           const HarmEntry* __restrict__ harm, float* __restrict__ chroma,
                                           float* __restrict__ energy, uint64_t g) {
#pragma unroll
        for (int q = 0; q < 12; q++) pc[q][i] = 0.0f;
#pragma unroll
        for (int k = 0; k < KCAP; k++) {
            if (k >= P.K || !(pm[k] > 0.0f)) continue;
            const int bin = pb[k];
            const float xk = sd_maxf(pm[k], 0.0f);
            float w0;
            if (P.p == 0.5f) {  // the default power: the correctly rounded sqrt where it is sd_powf's value
                const float s = __builtin_sqrtf(xk);
                w0 = sd_sqrt_is_powf_half(xk, s) ? s : sd_powf_ool(xk, 0.5f);
            } else {
                w0 = sd_powf_ool(xk, P.p);
            }
            if (w0 <= 0.0f) continue;
#ifdef SDSP_HPCP_DIAG_NOHARM
            pc[bin % 12][i] += w0;  // diagnostic timing build: no harmonic table walk (wrong chroma)
            continue;
#endif
#ifndef SDSP_HPCP_HARM_SEQ
            // the peak's first HU table entries (128 contiguous bytes) are loaded together, ahead of
            // their use, instead of one dependent load per harmonic; the accumulation order is the
            // same (h ascending, the walk ends at the first state-0 entry)
            HarmEntry hv[HU];
#pragma unroll
            for (int h = 0; h < HU; h++)
                if (h < P.hmax) hv[h] = harm[bin * HP_HMAX + h];
            bool stop = false;
#pragma unroll
            for (int h = 0; h < HU; h++) {
                if (stop || h >= P.hmax) break;
                const HarmEntry& he = hv[h];
                if (he.state == 0) {
                    stop = true;
                    break;
                }
                if (he.state == 1) continue;
                const float contrib = w0 * he.hw;
                for (int o = 0; o < 3; o++) pc[he.tc[o]][i] += contrib * he.wt[o];
            }
            for (int h = HU + 1; !stop && h <= P.hmax; h++) {
#else
            for (int h = 1; h <= P.hmax; h++) {
#endif
                const HarmEntry he = harm[bin * HP_HMAX + (h - 1)];
                if (he.state == 0) break;
                if (he.state == 1) continue;
                const float contrib = w0 * he.hw;
                for (int o = 0; o < 3; o++) pc[he.tc[o]][i] += contrib * he.wt[o];
            }
        }
        float nsq = 0.0f;
#pragma unroll
        for (int q = 0; q < 12; q++) nsq += pc[q][i] * pc[q][i];
        const float norm = __builtin_sqrtf(nsq);
#pragma unroll
        for (int q = 0; q < 12; q++) {
            float v = pc[q][i];
            if (norm > EPS) v /= norm;
            chroma[g * 12 + q] = v;
        }
        energy[g] = e;
    }
};

// 4 waves per SIMD: round 3 measured it 8 % faster than the 3-wave build (14.6 vs 15.9 ms per
// 256-track launch, then at 128 VGPRs with a 16-byte spill); with per-wave staging and the
// pitch-class scratch in its own LDS array the HPCP kernels take 112 VGPRs, no spill
#ifndef SDSP_HPCP_ATTR
#define SDSP_HPCP_ATTR __attribute__((amdgpu_waves_per_eu(4)))
#endif
// One thread per frame, HP_FRAMES frames per workgroup.  Bins are staged through LDS in
// HP_CW-column chunks (coalesced row segments) and each thread walks its frame's bins in
// order (HpcpFrame).  Each wave stages the rows of its own 64 frames, so no workgroup barrier
// holds the waves together per chunk (as k_hpcp_band).
template <int KCAP>
__global__ __launch_bounds__(HP_FRAMES) SDSP_HPCP_ATTR void k_hpcp(const float* __restrict__ mags,
                                                    const uint64_t* __restrict__ frame_pfx,
                                                    const uint64_t* __restrict__ tile_pfx,
                                                    const int* __restrict__ tracks, int n_items, HpcpParams P,
                                                    const HarmEntry* __restrict__ harm, float* __restrict__ chroma,
                                                    float* __restrict__ energy) {
    __shared__ float tile[HP_FRAMES][HP_CW + 1];
    __shared__ float pcs[12][HP_FRAMES];  // pitch-class accumulators (a column per thread)
    const uint64_t gb = blockIdx.x;
    const int it = find_track(tile_pfx, n_items, gb);
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[it]) * HP_FRAMES;
    const int i = threadIdx.x;
    const int64_t f = f0 + i;
    const bool valid = f < F;
    const int lane = i & 63, wrow = i & ~63;
    const int64_t rows = F - f0 < HP_FRAMES ? F - f0 : HP_FRAMES;
    if (wrow >= rows) return;  // the whole wave is past the track's end
    const uint64_t g0 = frame_pfx[trk];
    HpcpFrame<KCAP> hf;
    hf.init();
    constexpr int RSTEP = 64 / HP_CW;
    constexpr int NLD = 64 / RSTEP;
    const int sub = lane / HP_CW, jj = lane % HP_CW;
    // software pipeline: chunk c0+HP_CW is loaded into registers while chunk c0 is walked
    const float* rowp = mags + (g0 + (uint64_t)f0 + (uint64_t)(wrow + sub)) * (uint64_t)P.stride + jj;
    const uint64_t rstride = (uint64_t)RSTEP * (uint64_t)P.stride;
    float nx[NLD];
    auto load_chunk = [&](int c0) {
        const bool col_ok = c0 + jj < P.B;
#pragma unroll
        for (int u = 0; u < NLD; u++)
            nx[u] = (wrow + sub + u * RSTEP < rows && col_ok) ? rowp[(uint64_t)u * rstride + c0] : 0.0f;
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    load_chunk(0);
    for (int c0 = 0; c0 < P.B; c0 += HP_CW) {
        wave_sync();  // the previous chunk's walk has read its rows
#pragma unroll
        for (int u = 0; u < NLD; u++) tile[wrow + sub + u * RSTEP][jj] = nx[u];
        wave_sync();
        if (c0 + HP_CW < P.B) load_chunk(c0 + HP_CW);
        if (!valid) continue;
        hf.walk(tile[i], c0, P.B - c0 < HP_CW ? P.B - c0 : HP_CW, P);
    }
    if (!valid) return;
    hf.finish(pcs, i, P, harm, chroma, energy, g0 + (uint64_t)f);
}

// A rigorous bound on |e_blk - e_ref| / e_blk for one frame ("Certification"): e_blk
// is this engine's fold of the 65 block sums Bt_b (each an f32 fold of its 64 squares
// t_k = RN(x_k^2) from 0, k_mask_rp: two sequential halves of 32, then their sum; the g63 bound
// below holds for any association of 64 non-negative terms, since no term passes through more than
// 63 roundings), e_ref the reference's one sequential f32 fold of the same
// 4,097 squares (extractor.rs:1133).  With u = 2^-24, T = sum t_k (exact), B_b the exact block sums:
//   |Bt_b - B_b| <= g63 B_b, so B_b <= Bt_b / (1 - g63) =: Bu_b;
//   |e_blk - sum Bt_b| <= u (1 + g64) sum_b (Bt_0 + .. + Bt_b)   (one rounding per block fold step);
//   |sum Bt_b - T| <= g63 sum_b Bu_b;
//   |e_ref - T| <= sum_k |d_k|, d_k the rounding of the reference's step k: |d_k| <= t_k (its
//   partial sum S_{k-1} is a float next to S_{k-1} + t_k) and |d_k| <= u (1 + u) U_b for k in block
//   b, U_b = (Bu_0 + .. + Bu_b)(1 + gN) bounding every partial sum there (the terms are >= 0), so
//   block b adds at most min(Bu_b, n_b u (1 + u) U_b).
// Evaluated in double (relative error ~1e-14, covered by a 1e-9 factor) and rounded up to f32.
// e_blk = 0 means every square is +0, so both folds are +0 (bound 0).
__device__ float energy_delta(const float* __restrict__ pp, uint64_t total, int n_blocks, int B, float e_blk) {
    if (!(e_blk > 0.0f)) return 0.0f;
    const double u = 0x1p-24, g63 = 63.0 * u / (1.0 - 63.0 * u), g64 = 64.0 * u / (1.0 - 64.0 * u);
    const double gN = (double)B * u / (1.0 - (double)B * u), iu = 1.0 / (1.0 - g63);
    double pu = 0.0, pt = 0.0, eref = 0.0, eo = 0.0;
    for (int g = 0; g < n_blocks; g++) {
        const double bt = (double)pp[(uint64_t)g * total], bu = bt * iu;
        pu += bu;
        pt += bt;
        const int nb = B - 64 * g < 64 ? B - 64 * g : 64;
        eref += __builtin_fmin(bu, (double)nb * u * (1.0 + u) * pu * (1.0 + gN));
        eo += pt;
    }
    const double D = (eref + u * (1.0 + u) * (1.0 + g64) * eo + g63 * pu) * (1.0 + 1e-9);
    const double r = D / (double)e_blk;
    if (!(r < 1.0)) return 1.0f;  // no usable bound (cannot happen for finite sums); the vote flags it
    float d = (float)r;
    if ((double)d < r) d = __uint_as_float(__float_as_uint(d) + 1u);
    return d;
}

// energy_delta's bound from its terms accumulated in f32 (round 6): every term is >= 0 and every f32
// operation rounds to nearest, so each computed sum or product is at least (1 - 2^-24)^m of its exact
// value for the m <= 300 roundings on its path (the constants' included), and the computed bound
// times (1 + 2^-14) is an upper bound of the exact one (300 * 2^-24 = 1.8e-5 < 2^-14 = 6.1e-5, the
// final division's rounding included).  Outside e in [2^-60, 2^100] (no overflow; no denormal loses
// more than 2^-141 absolute against a bound >= 2^-78) the double evaluation runs instead.
constexpr float KC_IU_F = (float)(1.0 / (1.0 - 63.0 * 0x1p-24 / (1.0 - 63.0 * 0x1p-24)));
__device__ float energy_delta_f32(float e_blk, float pu, float eref, float eo, const float* __restrict__ pp,
                                  uint64_t total, int n_blocks, int B) {
    if (!(e_blk > 0.0f)) return 0.0f;
    if (!(e_blk >= 0x1p-60f && e_blk <= 0x1p100f)) return energy_delta(pp, total, n_blocks, B, e_blk);
    const float u = 0x1p-24f;
    const float g63 = 63.0f * u / (1.0f - 63.0f * u), g64 = 64.0f * u / (1.0f - 64.0f * u);
    const float D = eref + u * (1.0f + u) * (1.0f + g64) * eo + g63 * pu;
    const float r = (D / e_blk) * (1.0f + 0x1p-14f);
    if (!(r < 1.0f)) return 1.0f;  // no usable bound; the vote flags it
    return r;
}

// k_hpcp_band: k_hpcp after k_mask_rp.  The frame energy folds the 65 block sums part[g][frame] in
// block order; the bin walk covers only the band k_mask_rp stored, [pk_lo - 1, pk_hi + 1] (the
// local-maximum test of candidate c reads bins c - 1 .. c + 1; starting the walk at pk_lo - 1 with
// the walk's zero history gives exactly k_hpcp's candidates).  Each wave stages the 64 rows of its
// own frames, so the waves run without workgroup barriers: a wave whose frames insert more peaks
// does not hold the others at a barrier per chunk (a wave's LDS operations execute in order; a
// wave-level fence keeps the staging writes and the walk's reads in program order).
#ifndef SDSP_HPCP_BAND_HU
#define SDSP_HPCP_BAND_HU 4
#endif
template <int KCAP>
__global__ __launch_bounds__(HP_FRAMES) SDSP_HPCP_ATTR void k_hpcp_band(const float* __restrict__ mags,
                                                         const uint64_t* __restrict__ frame_pfx,
                                                         const uint64_t* __restrict__ tile_pfx,
                                                         const int* __restrict__ tracks, int n_items, HpcpParams P,
                                                         const HarmEntry* __restrict__ harm,
                                                         const float* __restrict__ part, int n_blocks, uint64_t total,
                                                         float* __restrict__ chroma, float* __restrict__ energy,
                                                         float* __restrict__ edel) {
    __shared__ float tile[HP_FRAMES][HPB_CW + 1];
    __shared__ float pcs[12][HP_FRAMES];  // pitch-class accumulators (a column per thread)
    const uint64_t gb = blockIdx.x;
    const int it = find_track(tile_pfx, n_items, gb);
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[it]) * HP_FRAMES;
    const int i = threadIdx.x;
    const int64_t f = f0 + i;
    const bool valid = f < F;
    const int lane = i & 63, wrow = i & ~63;
    const int64_t rows = F - f0 < HP_FRAMES ? F - f0 : HP_FRAMES;
    if (wrow >= rows) return;  // the whole wave is past the track's end
    const uint64_t g0 = frame_pfx[trk];
    HpcpFrame<KCAP> hf;
    hf.init();
    if (valid) {
        const float* pp = part + g0 + (uint64_t)f;
#ifndef SDSP_HPCP_EDEL_DOUBLE
        // the frame energy (pt: the block sums folded in block order) and, in the same pass, the
        // certificate's bound terms in f32 (energy_delta_f32)
        const float u = 0x1p-24f;
        const float gN = (float)P.B * u / (1.0f - (float)P.B * u);
        const float c64 = 64.0f * u * (1.0f + u) * (1.0f + gN);
        const float clast = (float)(P.B - 64 * (n_blocks - 1)) * u * (1.0f + u) * (1.0f + gN);
        float pt = 0.0f, pu = 0.0f, eref = 0.0f, eo = 0.0f;
        for (int g = 0; g < n_blocks; g++) {
            const float bt = pp[(uint64_t)g * total];
            pt += bt;
            const float bu = bt * KC_IU_F;
            pu += bu;
            eref += __builtin_fminf(bu, (g + 1 < n_blocks ? c64 : clast) * pu);
            eo += pt;
        }
        hf.e = pt;
        if (edel) edel[g0 + (uint64_t)f] = energy_delta_f32(pt, pu, eref, eo, pp, total, n_blocks, P.B);
#else
        float e = 0.0f;
        for (int g = 0; g < n_blocks; g++) e += pp[(uint64_t)g * total];
        hf.e = e;
        // the certificate's per-frame energy bound (k_key_vote, KeyParams::near_check)
        if (edel) edel[g0 + (uint64_t)f] = energy_delta(pp, total, n_blocks, P.B, e);
#endif
    }
    const int w_lo = P.pk_lo - 1 > 0 ? P.pk_lo - 1 : 0, w_hi = P.pk_hi + 1 < P.B - 1 ? P.pk_hi + 1 : P.B - 1;
    // lane (r4, q4) stages bins 4 q4 .. 4 q4 + 3 of rows wrow + r4 + 16 u (u < 4), one 16-byte load
    // per row: a wave load covers 16 rows' 64-byte segments (4 with 4-byte loads: 8.8 % slower per
    // launch, round 5)
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int r4 = lane >> 2, q4 = lane & 3;
    const f4v* rowp4 = reinterpret_cast<const f4v*>(mags + (g0 + (uint64_t)f0 + (uint64_t)(wrow + r4)) * (uint64_t)P.stride + 4 * q4);
    const uint64_t rstride4 = 4 * (uint64_t)P.stride;  // 16 rows, in f4v units
    f4v n4[4];
    auto load_chunk = [&](int c0) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            // a group wholly past w_hi is not read; one that starts at a bin b <= w_hi < B ends
            // inside the row (strides are multiples of 4 floats, at least B: b + 4 <= stride)
            const int b = c0 + 4 * q4;
            f4v v = {0.0f, 0.0f, 0.0f, 0.0f};
            if (wrow + r4 + 16 * u < rows && b <= w_hi) v = rowp4[(uint64_t)u * rstride4 + (uint64_t)(c0 >> 2)];
            n4[u] = f4v{b <= w_hi ? v.x : 0.0f, b + 1 <= w_hi ? v.y : 0.0f, b + 2 <= w_hi ? v.z : 0.0f,
                        b + 3 <= w_hi ? v.w : 0.0f};
        }
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // chunks on HPB_CW-bin boundaries, so every 64-byte row segment is one aligned sector (rows
    // are 64-byte aligned); the bins below w_lo this adds are no candidates (c < pk_lo), they only
    // pass through the walk's two-bin history.  (From w_lo itself: 2.2-2.5 % slower; the chunk after
    // next in flight too: 20-25 % slower, at 4 waves with spills or at 3; round 5.)
    const int c_start = w_lo & ~(HPB_CW - 1);
    if (w_lo <= w_hi) load_chunk(c_start);
    for (int c0 = c_start; c0 <= w_hi; c0 += HPB_CW) {
        wave_sync();  // the previous chunk's walk has read its rows
#pragma unroll
        for (int u = 0; u < 4; u++) {
            float* tr = tile[wrow + r4 + 16 * u] + 4 * q4;
            tr[0] = n4[u].x;
            tr[1] = n4[u].y;
            tr[2] = n4[u].z;
            tr[3] = n4[u].w;
        }
        wave_sync();
        if (c0 + HPB_CW <= w_hi) load_chunk(c0 + HPB_CW);
        if (!valid) continue;
        hf.template walk<false>(tile[i], c0, w_hi + 1 - c0 < HPB_CW ? w_hi + 1 - c0 : HPB_CW, P);
    }
    if (!valid) return;
    hf.template finish<SDSP_HPCP_BAND_HU>(pcs, i, P, harm, chroma, energy, g0 + (uint64_t)f);
}

// ----------------------------------------------------------------------------------------
// KeyParams::near_check: whether a weight perturbation of the size the block-folded energies make
// could change one of key_from_raw's discrete decisions on these raw scores: the within-mode
// argmax (a top-two gap of at most KV_NEAR_CONF relative) or the normalisation guard.  The argmax
// is what fixes the winners' normalised scores (exactly 1 each), so ties between the final
// winners are exact and stay exact while these decisions hold.
__device__ bool key_raw_near(const float raw[24]) {
    bool near = false;
    for (int m = 0; m < 2; m++) {
        float t1 = 0.0f, t2 = 0.0f;  // the fold keeps 0 as the floor, as key_from_raw's max does
        for (int k = 0; k < 12; k++) {
            const float v = raw[12 * m + k];
            if (v > t1) {
                t2 = t1;
                t1 = v;
            } else if (v > t2) {
                t2 = v;
            }
        }
        near |= t1 > 0.0f && !(t1 - t2 > KV_NEAR_CONF * t1);
        near |= sd_absf(t1 - 1e-9f) <= KV_NEAR_REL * 1e-9f;
    }
    return near;
}

__device__ void key_from_raw(const float raw[24], float sorted[24], int order[24]) {
    float sc[24];
    for (int k = 0; k < 24; k++) sc[k] = raw[k];
    float mM = 0.0f, mm = 0.0f;
    for (int k = 0; k < 12; k++) mM = sd_maxf(mM, sc[k]);
    for (int k = 0; k < 12; k++) mm = sd_maxf(mm, sc[12 + k]);
    if (mM > 1e-9f && mm > 1e-9f) {
        for (int k = 0; k < 12; k++) sc[k] /= mM;
        for (int k = 0; k < 12; k++) sc[12 + k] /= mm;
    }
    int tM = 0, tm = 0;
    for (int k = 1; k < 12; k++)
        if (!(sc[k] < sc[tM])) tM = k;
    for (int k = 1; k < 12; k++)
        if (!(sc[12 + k] < sc[12 + tm])) tm = k;
    const float tMs = sc[tM], tms = sc[12 + tm];
    const int cof_pos[12] = {0, 7, 2, 9, 4, 11, 6, 1, 8, 3, 10, 5};  // position of tonic on the circle
    float rs[24];
    for (int k = 0; k < 24; k++) {
        rs[k] = sc[k];
        const bool major = k < 12;
        const int ref_t = major ? tM : tm;
        const float ref_s = major ? tMs : tms;
        if (ref_s > 1e-9f) {
            const int tp = cof_pos[k % 12], rp = cof_pos[ref_t];
            const int ad = tp > rp ? tp - rp : rp - tp;
            const int dist = ad < 12 - ad ? ad : 12 - ad;
            if (dist <= 2) rs[k] += ref_s * (0.20f * (1.0f - (float)dist * 0.5f));
        }
    }
    for (int k = 0; k < 24; k++) order[k] = k;
    for (int a = 1; a < 24; a++) {  // stable insertion sort, desc
        const int o = order[a];
        int b = a;
        while (b > 0 && rs[order[b - 1]] < rs[o]) {
            order[b] = order[b - 1];
            b--;
        }
        order[b] = o;
    }
    for (int k = 0; k < 24; k++) sorted[k] = rs[order[k]];
}

__device__ float clarity_of(const float* s) {
    const float best = s[0];
    float sum = 0.0f;
    for (int i = 0; i < 24; i++) sum += s[i];
    const float avg = sum / 24.0f;
    float mn = s[0], mx = s[0];
    for (int i = 1; i < 24; i++) {
        if (s[i] < mn) mn = s[i];
        if (!(s[i] < mx)) mx = s[i];
    }
    const float range = mx - mn;
    return range > 1e-10f ? sd_clampf((best - avg) / range, 0.0f, 1.0f) : 0.0f;
}

// cof_pos above maps a tonic to its circle-of-fifths position: the reference searches
// circle_of_fifths = [0,7,2,9,4,11,6,1,8,3,10,5] for the tonic (detector.rs:214-224); that
// array is its own inverse, so position(t) = circle_of_fifths[t].

// stable sort desc of a 24-entry score table by key index, (best - second) / best
__device__ void from_table(const float* acc, float sorted[24], int order[24], float* conf) {
    for (int k = 0; k < 24; k++) order[k] = k;
    for (int a = 1; a < 24; a++) {
        const int o = order[a];
        int b = a;
        while (b > 0 && acc[order[b - 1]] < acc[o]) {
            order[b] = order[b - 1];
            b--;
        }
        order[b] = o;
    }
    for (int k = 0; k < 24; k++) sorted[k] = acc[order[k]];
    *conf = sorted[0] > 0.0f ? sd_clampf((sorted[0] - sorted[1]) / sorted[0], 0.0f, 1.0f) : 0.0f;
}

// detect_key_weighted_mode_heuristic on a base result (detector.rs:326-506): sorted/order become
// the post-bonus table (stable re-sort of the base order), *chosen the possibly mode-flipped key
// index (mode * 12 + tonic) and *conf its confidence.  avg_in: the raw weighted chroma sums,
// wsum: their weight total.
__device__ void mode_heuristic(float sorted[24], int order[24], const float* avg_in, float wsum, const KeyParams& P,
                               int* chosen, float* conf) {
    *chosen = order[0];
    *conf = sorted[0] > 0.0f ? sd_clampf((sorted[0] - sorted[1]) / sorted[0], 0.0f, 1.0f) : 0.0f;
    const float flip_ratio = sd_clampf(P.mh_flip, 0.0f, 1.0f);
    const bool mode_flip = flip_ratio > 0.0f;
    if (!P.mh_bonus && !mode_flip) return;
    if (wsum <= 1e-9f) return;
    float avg[12];
    float sum = -0.0f;
    for (int i = 0; i < 12; i++) {
        avg[i] = avg_in[i];
        sum += avg[i];
    }
    if (sum > 1e-9f)
        for (int i = 0; i < 12; i++) avg[i] /= sum;
    if (P.mh_bonus) {
        const float bw = sd_maxf(P.mh_bonus_w, 0.0f);
        if (bw > 0.0f)
            for (int i = 0; i < 24; i++)
                if (order[i] >= 12) {
                    const int tonic = order[i] - 12;
                    sorted[i] += wsum * bw * (avg[(tonic + 11) % 12] - avg[(tonic + 10) % 12]);
                }
    }
    for (int a = 1; a < 24; a++) {  // stable insertion sort of the base-ordered table, desc
        const float v = sorted[a];
        const int o = order[a];
        int b = a;
        while (b > 0 && sorted[b - 1] < v) {
            sorted[b] = sorted[b - 1];
            order[b] = order[b - 1];
            b--;
        }
        sorted[b] = v;
        order[b] = o;
    }
    float maj_s[12], min_s[12];
    for (int i = 0; i < 24; i++) {
        if (order[i] < 12)
            maj_s[order[i]] = sorted[i];
        else
            min_s[order[i] - 12] = sorted[i];
    }
    const int best = order[0], tonic = best % 12;
    const bool best_major = best < 12;
    const float p_min3 = avg[(tonic + 3) % 12], p_maj3 = avg[(tonic + 4) % 12];
    const float p_min6 = avg[(tonic + 8) % 12], p_maj6 = avg[(tonic + 9) % 12];
    const float p_min7 = avg[(tonic + 10) % 12], p_maj7 = avg[(tonic + 11) % 12];
    const float margin = sd_maxf(P.mh_margin, 0.0f);
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
    int ch = best;
    if (mode_flip) {
        if (best_major && minor_pref) {
            if (maj_s[tonic] > 0.0f && min_s[tonic] >= maj_s[tonic] * flip_ratio) ch = 12 + tonic;
        } else if (!best_major && major_pref) {
            if (min_s[tonic] > 0.0f && maj_s[tonic] >= min_s[tonic] * flip_ratio) ch = tonic;
        }
    }
    const float cs = ch < 12 ? maj_s[ch] : min_s[ch - 12];
    float other = 0.0f;
    for (int i = 0; i < 24; i++)
        if (order[i] != ch) other = sd_maxf(other, sorted[i]);
    *chosen = ch;
    *conf = cs > 0.0f ? sd_clampf((cs - other) / cs, 0.0f, 1.0f) : 0.0f;
}

constexpr int KV_MAXSCALE = 8;

// ---- the rigorous near-decision certificate (KeyParams::near_check, cert_fixed = 0) ----
// k_hpcp_band bounds each frame's energy by |e_ref - e| <= d_f e (energy_delta).  With p the energy
// power, the reference's frame weight is w'_f = c w_f (1 + eps_f), |eps_f| <= eta_f (kc_eta), c the
// factor (med / med')^p its median carries for every frame alike: every decision below is invariant
// under a common factor of the weights, so only eta_f and the roundings matter.  Every raw score is
// R_x = sequential sum over frames of RN(w_f D_fx) (D_fx the frame's template dot, identical on both
// sides), so |R'_x - c R_x| <= c (V_x (1 + 2u) + N_x) with V_x = sum_f eta_f w_f D_fx and
// N_x = u (2.0001 R_x + (1 + K) SS_x), SS_x the sum of the fold's partial sums (both sides' roundings;
// K bounds the reference's partial sums against c times ours).
constexpr double KC_U = 0x1p-24;
constexpr int KC_CAP = 32;
struct KcCand {
    int64_t st;     // the table's frames [st, st + len) of the slice
    int len, w, k;  // the mode's argmax W and a competitor k (key indices)
    float slack;    // G - N_W - N_k - 1.01 u R_W: what E_Wk must stay below
};
// a non-negative double rounded up to f32
__device__ __forceinline__ float kc_up(double x) {
    float d = (float)x;
    if ((double)d < x) d = __uint_as_float(__float_as_uint(d) + 1u);
    return d;
}
__device__ __forceinline__ double kc_noise(double R, double SS, double K) { return KC_U * (2.0001 * R + (1.0 + K) * SS); }
// eta_f for an energy bound d and energy power p: the weight ratio w'/(c w) lies in [e^-L, e^L] with
// L = p d / (1 - d) (the energy) + 2.0001 u p (the two e / med roundings) + 2.0001 (u + 2^-40) (the
// two powf evaluations: double exp / log, then one rounding) + 2.0001 u (the two tonal products);
// e^L - 1 <= L / (1 - L)
__device__ __forceinline__ double kc_eta(double d, double p) {
    const double L = p * d / (1.0 - d) + 2.0001 * KC_U * p + 2.0001 * (KC_U + 0x1p-40) + 2.0001 * KC_U;
    return L / (1.0 - L);
}
// The within-mode argmaxes (key_from_raw's last maximum W) of the reference equal this table's when,
// for every other key k of the mode, G = R_W - R_k > N_W + N_k + E_Wk + 1.01 u R_W (the margin keeps
// RN(R'_k / R'_W) below 1, so the normalised scores cannot tie), where E_Wk = sum_f eta_f w_f
// |D_fW - D_fk| <= V_W + V_k.  Pairs that fail even with E_Wk = 0 are flagged; pairs that only the
// loose V_W + V_k fails are queued for the pair pass (kc_pair_pass), which computes E_Wk.
__device__ __noinline__ int kc_argmax(const float* raw, const float* SS, const float* V, double sf, double K, int64_t st, int len,
                         KcCand* list, int* nlist) {
    int bits = 0;
    for (int m = 0; m < 2; m++) {
        int W = 0;
        for (int k = 1; k < 12; k++)
            if (!(raw[12 * m + k] < raw[12 * m + W])) W = k;
        const double RW = raw[12 * m + W];
        if (!(RW > 0.0)) continue;  // an all-zero mode: every product is +0 on both sides
        const double NW = kc_noise(RW, SS[12 * m + W] * sf, K), VW = V[12 * m + W] * sf;
        for (int k = 0; k < 12; k++) {
            if (k == W) continue;
            const double Rk = raw[12 * m + k], G = RW - Rk;
            const double need0 = NW + kc_noise(Rk, SS[12 * m + k] * sf, K) + 1.01 * KC_U * RW;
            if (G > need0 + (VW + V[12 * m + k] * sf) * (1.0 + 2.0001 * KC_U)) continue;
            const int q = G > need0 ? atomicAdd(nlist, 1) : KC_CAP;
            if (q < KC_CAP) {
                float sl = (float)(G - need0);
                if ((double)sl > G - need0) sl = __uint_as_float(__float_as_uint(sl) - 1u);  // round down
                list[q] = KcCand{st, len, 12 * m + W, 12 * m + k, sl};
            } else {
                bits |= KV_NEAR_ARGMAX;
            }
        }
    }
    return bits;
}
// The clarity gate of one segment (src/lib.rs:1379-1380, key_clarity.rs:51-93), given that both
// within-mode argmaxes hold (kc_argmax): each mode's top is normalised to exactly 1 and gets the
// same bonus on both sides, so best = RN(1 + 0.2f) exactly, and every other post-bonus score rs_x
// moves by at most beta_x = B_x + 2.0001 u (sc_x + rs_x), B_x = (A_x + sc_x A_W) / (R_W - A_W)
// bounding |R'_x / R'_W - R_x / R_W| (A_x = V_x (1 + 2u) + N_x).  The sum over the sorted table
// (whose order may differ) moves by sum beta + 2 * 23 u sum rs, the minimum by max beta, and
// clarity = (best - avg) / (best - min) by the returned bound.  beta_x is written per key.
__device__ __noinline__ double kc_clarity(const float* raw, const float* SS, const float* V, double sf, double K, const float* sorted,
                             const int* order, float* beta, int* bits) {
    auto Ax = [&](int x) { return V[x] * sf * (1.0 + 2.0001 * KC_U) + kc_noise(raw[x], SS[x] * sf, K); };
    int Wm[2];
    double AW[2];
    for (int m = 0; m < 2; m++) {
        int W = 0;
        for (int k = 1; k < 12; k++)
            if (!(raw[12 * m + k] < raw[12 * m + W])) W = k;
        Wm[m] = 12 * m + W;
        AW[m] = Ax(Wm[m]);
        // the normalisation guard (max > 1e-9, detector.rs:165) with the common factor's range is
        // checked by the caller; here an unnormalised table is simply not certified
        if (!(raw[Wm[m]] > 1e-9f) || !((double)raw[Wm[m]] - AW[m] > 0.0)) {
            *bits |= KV_NEAR_RANGE;
            return 1.0;
        }
    }
    double sb = 0.0, bmax = 0.0;
    for (int i = 0; i < 24; i++) {
        const int x = order[i];
        const int W = Wm[x / 12];
        double b = 0.0;
        if (x != W) {
            const double M = raw[W], sc = (double)raw[x] / M, aw = AW[x / 12];
            b = (Ax(x) + sc * aw) / (M - aw) + 2.0001 * KC_U * (sc + (double)sorted[i]);
        }
        beta[x] = kc_up(b);
        sb += b;
        bmax = b > bmax ? b : bmax;
    }
    double srs = 0.0, mn = sorted[0];
    for (int i = 0; i < 24; i++) {
        srs += (double)sorted[i];
        mn = (double)sorted[i] < mn ? (double)sorted[i] : mn;
    }
    const double best = sorted[0], range = best - mn, avg = srs / 24.0, num = best - avg;
    const double dsum = sb + 2.0 * 23.0 * KC_U * srs * 1.01;
    const double davg = dsum / 24.0 + 2.0 * KC_U * __builtin_fabs(avg) * 1.01;
    const double dnum = davg + 2.0 * KC_U * __builtin_fabs(num) * 1.01;
    const double drange = bmax + 2.0 * KC_U * range * 1.01;
    if (!(range - drange > 1e-6)) {
        *bits |= KV_NEAR_RANGE;
        return 1.0;
    }
    const double cl0 = __builtin_fabs(num / range);
    return (dnum + cl0 * drange) / (range - drange) + 2.0 * KC_U * cl0 * 1.01 + 1e-15;
}

// threads per track in k_key_vote.  1024 halves the kernel's serial time (its frame loops are
// latency-bound) but triples it in the two-stream pipeline (16.9 vs 5.5 ms per launch): a
// 1024-thread workgroup needs most of a CU's VGPRs at once, and beside the 8192-point STFT's
// 256-VGPR waves such a CU seldom comes free
#ifndef KV_THREADS
#define KV_THREADS 256
#endif
#ifndef KV_SMALL_ITEMS
#define KV_SMALL_ITEMS 96
#endif
#ifdef SDSP_KV_PROF
#define KV_T(i) do { if (threadIdx.x == 0) kv_t[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define KV_T(i) do { } while (0)
#endif
template <int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_key_vote(const int* __restrict__ tracks, int n_items,
                                                  const uint64_t* __restrict__ frame_pfx, float* __restrict__ chroma_raw,
                                                  const float* __restrict__ energy, float* __restrict__ chroma_s,
                                                  float* __restrict__ weights, float* __restrict__ seg_scratch,
                                                  const uint64_t* __restrict__ seg_off, const float* __restrict__ tmpl,
                                                  KeyParams P, KeyOut* __restrict__ out, KeyDbg* __restrict__ dbg,
                                                  const float* __restrict__ edel, float* __restrict__ wdel) {
    __shared__ int hist[256];
    __shared__ int misc[4];
    __shared__ int redi[NT / 64];
    __shared__ float acc[48];
    __shared__ int use_w_s, used_s, near_s;
    __shared__ float totw_s;
    __shared__ float tpl[48][12];
    __shared__ int sc_len[KV_MAXSCALE], sc_pfx[KV_MAXSCALE + 1];
    __shared__ float sc_w[KV_MAXSCALE];
    // the certificate (cert): argmax pairs for the pair pass, the slice's largest energy bound and
    // eta, per-key vote bounds, the full slice's partial-sum totals and sensitivities
    __shared__ KcCand kc_list[KC_CAP];
    __shared__ int kc_n;
    __shared__ unsigned int kc_dmax, kc_emax;
    __shared__ float kc_pa[24], kc_ss[24], kc_v[24];
    __shared__ int kc_w;
    __shared__ double kc_red[NT / 64];
    __shared__ float kc_crs;  // the common factor's relative range (the median's), for absolute thresholds
    const bool cert = P.near_check && !P.cert_fixed && edel && wdel;
#ifdef SDSP_KV_PROF
    uint64_t kv_t[12] = {};
#endif
    KV_T(0);
    const int it = blockIdx.x;
    const int trk = tracks[it];
    const int64_t F_all = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const uint64_t g0 = frame_pfx[trk];
    float* cr = chroma_raw + g0 * 12;
    for (int k = threadIdx.x; k < 576; k += blockDim.x) tpl[k / 12][k % 12] = tmpl[k];
    if (threadIdx.x == 0) {  // published by the barriers below before any reader
        near_s = 0;
        kc_n = 0;
        kc_dmax = 0u;
        kc_emax = 0u;
    }
    if (F_all <= 0) {
        if (threadIdx.x == 0) out[trk] = KeyOut{0, 0, 0.0f, 0.0f, 0, 0, 0, 0};
        return;
    }
    // chroma sharpening (src/lib.rs:1200-1208 -> chroma/normalization.rs:41-65), in place
    if (P.sharpen > 1.0f) {
        for (int64_t f = threadIdx.x; f < F_all; f += blockDim.x) {
            float* c = cr + f * 12;
            float sq = 0.0f;
            for (int i = 0; i < 12; i++) {
                c[i] = sd_powf(c[i], P.sharpen);
                sq += c[i] * c[i];
            }
            const float nrm = __builtin_sqrtf(sq);
            if (nrm > 1e-10f) {
                for (int i = 0; i < 12; i++) c[i] /= nrm;
            } else {
                const float u = 1.0f / __builtin_sqrtf(12.0f);
                for (int i = 0; i < 12; i++) c[i] = u;
            }
        }
        __syncthreads();
    }
    // median smoothing, window 5 (src/lib.rs:1211-1213 -> smoothing.rs:37-94)
    float* cs_all = chroma_s + g0 * 12;
    // interior frames: the 5 values sorted by odd-even transposition (adjacent compare-exchanges
    // that swap only when the later value is strictly smaller: a stable sort, so its output equals
    // the insertion sort's element for element), branch-free; the edges keep the insertion sort
    auto cx = [](float& a, float& b) {
        const bool sw = b < a;
        const float lo = sw ? b : a, hi = sw ? a : b;
        a = lo;
        b = hi;
    };
    for (int64_t q = threadIdx.x; q < F_all * 12; q += blockDim.x) {
        const int64_t f = (int64_t)((uint32_t)q / 12u);  // F_all * 12 < 2^32
        const int s = (int)((uint32_t)q - 12u * (uint32_t)f);
        if (F_all > 5 && f >= 2 && f + 2 < F_all) {
            const float* c = cr + (f - 2) * 12 + s;
            float v0 = c[0], v1 = c[12], v2 = c[24], v3 = c[36], v4 = c[48];
#pragma unroll
            for (int r = 0; r < 5; r++) {
                if (r % 2 == 0) {
                    cx(v0, v1);
                    cx(v2, v3);
                } else {
                    cx(v1, v2);
                    cx(v3, v4);
                }
            }
            cs_all[q] = v2;
        } else if (F_all > 5) {
            float v[5];
            int n = 0;
            for (int o = -2; o <= 2; o++) {
                const int64_t fi = f + o;
                if (fi >= 0 && fi < F_all) v[n++] = cr[fi * 12 + s];
            }
            for (int a = 1; a < n; a++) {
                const float x = v[a];
                int b = a;
                while (b > 0 && x < v[b - 1]) {
                    v[b] = v[b - 1];
                    b--;
                }
                v[b] = x;
            }
            cs_all[q] = v[n / 2];
        } else {
            cs_all[q] = cr[q];
        }
    }
    __syncthreads();
    KV_T(1);
    // optional edge trim (src/lib.rs:1215-1232): keep the middle frames
    int64_t t0 = 0, F = F_all;
    if (P.edge_trim && F_all >= 200) {
        const float frac = sd_clampf(P.edge_frac, 0.0f, 0.49f);
        const int64_t st = (int64_t)sd_roundf((float)F_all * frac);
        const int64_t en_ = (int64_t)sd_roundf((float)F_all * (1.0f - frac));
        if (en_ > st + 50 && en_ <= F_all) {
            t0 = st;
            F = en_ - st;
        }
    }
    const float* cs = cs_all + t0 * 12;
    const float* en = energy + g0 + t0;
    float* w = weights + g0 + t0;
    const float* ed = cert ? edel + g0 + t0 : nullptr;
    float* wd = cert ? wdel + g0 + t0 : nullptr;
    // frame weights over the slice (src/lib.rs:1236-1287)
    if (P.weighting) {
        const float med = sd_maxf(block_select_kth(en, (int)F, (int)(F / 2), hist, misc), 1e-12f);
        const float ln12 = sd_logf(12.0f);
        int used_local = 0, rng_local = 0;
        uint32_t dmax_local = 0u, emax_local = 0u;
        for (int64_t f = threadIdx.x; f < F; f += blockDim.x) {
            const float* ch = cs + f * 12;
            float sum = 0.0f;
            for (int k = 0; k < 12; k++) sum += ch[k];
            float tonal = 0.0f;
            if (!(sum <= 1e-12f)) {
                float ent = 0.0f;
                for (int k = 0; k < 12; k++) {
                    const float p = ch[k] / sum;
                    if (p > 1e-12f) ent -= p * sd_logf(p);
                }
                tonal = sd_clampf(1.0f - (ent / ln12), 0.0f, 1.0f);
            }
            if (tonal < P.min_tonal) tonal = 0.0f;
            const float e_norm = sd_maxf(en[f] / med, 0.0f);
            const float wt = sd_powf(tonal, sd_maxf(P.tonal_pow, 0.0f));
            const float we = sd_powf(e_norm, sd_maxf(P.energy_pow, 0.0f));
            const float ww = sd_maxf(wt * we, 0.0f);
            w[f] = ww;
            used_local += ww > 0.0f;
            if (cert) {  // eta_f w_f, and the range the certificate assumes
                const double d = ed[f];
                const double eta = d < 0.25 ? kc_eta(d, sd_maxf(P.energy_pow, 0.0f)) : 1.0;
                wd[f] = ww > 0.0f ? kc_up(eta * (double)ww) : 0.0f;
                // an energy whose quotient or weight could underflow on one side only, or no bound
                if (!(d < 0.25) || (en[f] > 0.0f && !(e_norm >= 0x1p-100f) && we != 1.0f) ||
                    (ww > 0.0f && !(ww >= 0x1p-100f)) || !(ww < 0x1p100f))
                    rng_local = 1;
                dmax_local = max(dmax_local, __float_as_uint((float)d));
                emax_local = max(emax_local, __float_as_uint(kc_up(eta)));
            }
        }
        if (cert) {  // one LDS atomic per wave (the maxima of non-negative floats as bit patterns)
            const uint32_t dm = wave_max_u32(dmax_local), em = wave_max_u32(emax_local);
            const bool rg = __builtin_amdgcn_ballot_w64(rng_local != 0) != 0;
            if ((threadIdx.x & 63) == 0) {
                if (rg) atomicOr(&near_s, KV_NEAR_RANGE);
                atomicMax(&kc_dmax, dm);
                atomicMax(&kc_emax, em);
            }
        }
        const int used = block_sum_i(used_local, redi);
        __syncthreads();
        __shared__ float sbuf[SEQ_CH];
        const float sw = block_seq_sum(w, F, sbuf);  // weights.iter().sum(), in order
        if (threadIdx.x == 0) {
            use_w_s = !(sw <= 1e-12f || used < 10);
            // the unweighted fallback (src/lib.rs:1278-1285) is decided by a sum of energy-derived weights:
            // sw' = c sw (1 +- eta_max) +- both folds' roundings, c in [(1 + d_max)^-p, (1 - d_max)^-p]
            float mrel = KV_NEAR_REL;
            if (cert) {
                const double dm = __uint_as_float(kc_dmax), em = __uint_as_float(kc_emax);
                const double L = sd_maxf(P.energy_pow, 0.0f) * dm / (1.0 - dm);
                const double cr = (L < 0.5 ? L / (1.0 - L) : 1.0);
                kc_crs = kc_up(cr);
                mrel = sd_maxf(mrel, kc_up(((1.0 + cr) * (1.0 + em) * (1.0 + 3.0 * (double)F * KC_U) - 1.0) * 1.01));
            }
            if (P.near_check && sd_absf(sw - 1e-12f) <= mrel * 1e-12f) atomicOr(&near_s, KV_NEAR_WSUM);
        }
    } else if (threadIdx.x == 0) {
        use_w_s = 0;
    }
    __syncthreads();
    KV_T(2);
    const bool use_w = use_w_s;
    const int toff = P.tset == 1 ? 24 : 0;  // template rows of the selected set
    if (dbg) {  // debug_track_id: weighted pitch-class sums over the slice, in frame order (src/lib.rs:1473-1491)
        if (threadIdx.x < 12) {
            float a = 0.0f;
            for (int64_t f = 0; f < F; f++) {
                const float wt = use_w ? w[f] : 1.0f;
                if (wt <= 0.0f) continue;
                a += wt * cs[f * 12 + threadIdx.x];
            }
            acc[threadIdx.x] = a;
        }
        if (threadIdx.x == 32) {
            int u = 0;
            for (int64_t f = 0; f < F; f++) u += (use_w ? w[f] : 1.0f) > 0.0f;
            dbg[it].frames = (int)F;
            dbg[it].used = u;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            float sa = 0.0f;
            for (int k = 0; k < 12; k++) sa += acc[k];
            for (int k = 0; k < 12; k++) dbg[it].agg[k] = sa > 1e-12f ? acc[k] / sa : acc[k];
        }
        __syncthreads();
    }
    // the final score table for the debug dump (KeyDetectionResult::top_keys)
    auto put_dbg = [&](const float* sorted, const int* order, int key) {
        if (!dbg) return;
        for (int k = 0; k < 24; k++) {
            dbg[it].tab[k] = sorted[k];
            dbg[it].order[k] = order[k];
        }
        dbg[it].key = key;
    };
    // Both folds below skip frames of weight <= 0 (detector.rs:992, 351).  Every term is >= +0
    // (chroma, templates and weights are non-negative), so a skipped frame is folded as +0, which
    // leaves the sum bit-identical; the loops then carry no branch and their loads pipeline
    // across frames.
    auto wsd = [&](int64_t f0, int64_t n, int row) {  // weighted_sum_dot, detector.rs:984-1001
        float a = 0.0f;
        const float* t = tpl[row];
        float tr[12];
#pragma unroll
        for (int k = 0; k < 12; k++) tr[k] = t[k];
#pragma unroll 4
        for (int64_t f = f0; f < f0 + n; f++) {
            const float* c = cs + f * 12;
            float d = 0.0f;
#pragma unroll
            for (int k = 0; k < 12; k++) d += c[k] * tr[k];
            if (use_w) {
                const float wt = w[f];
                a += wt > 0.0f ? wt * d : 0.0f;
            } else {
                a += d;
            }
        }
        return a;
    };
    // weighted_sum_dot with the certificate's companions: *ss = the sum of the fold's partial sums,
    // *vv = sum_f eta_f w_f D_f (f32 sums of non-negative terms; the readers inflate them by (n + 1) u)
    auto wsd3 = [&](int64_t f0, int64_t n, int row, float* ss, float* vv) {
        float a = 0.0f, sa = 0.0f, v = 0.0f;
        const float* t = tpl[row];
        float tr[12];
#pragma unroll
        for (int k = 0; k < 12; k++) tr[k] = t[k];
#pragma unroll 4
        for (int64_t f = f0; f < f0 + n; f++) {
            const float* c = cs + f * 12;
            float d = 0.0f;
#pragma unroll
            for (int k = 0; k < 12; k++) d += c[k] * tr[k];
            const float wt = w[f];
            a += wt > 0.0f ? wt * d : 0.0f;
            sa += a;
            v = __builtin_fmaf(wd[f], d, v);
        }
        *ss = sa;
        *vv = v;
        return a;
    };
    // the certificate's inflation of those f32 sums, and K (kc_noise) for a table of n frames
    auto kc_sf = [](int64_t n) { return 1.0 + 1.0001 * (double)(n + 1) * KC_U; };
    auto kc_K = [&](int64_t n) { return (1.0 + (double)__uint_as_float(kc_emax)) * (1.0 + 3.0 * (double)n * KC_U); };
    // the pair pass (kc_argmax's queue): E_Wk = sum_f eta_f w_f |D_fW - D_fk| over the pair's frames
    // by the whole workgroup, in double; a pair is certified when E_Wk (1 + 1e-6) < its slack
    auto kc_pair_pass = [&]() {
        __syncthreads();
        const int nc = kc_n < KC_CAP ? kc_n : KC_CAP;
        for (int q = 0; q < nc; q++) {
            const KcCand cd = kc_list[q];
            const float* tW = tpl[toff + cd.w];
            const float* tK = tpl[toff + cd.k];
            double e = 0.0;
            for (int64_t f = cd.st + threadIdx.x; f < cd.st + cd.len; f += blockDim.x) {
                const float wf = wd[f];
                if (!(wf > 0.0f)) continue;
                const float* c = cs + f * 12;
                float dW = 0.0f, dK = 0.0f;
#pragma unroll
                for (int k = 0; k < 12; k++) dW += c[k] * tW[k];
#pragma unroll
                for (int k = 0; k < 12; k++) dK += c[k] * tK[k];
                e += (double)wf * __builtin_fabs((double)dW - (double)dK);
            }
            for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
            if ((threadIdx.x & 63) == 0) kc_red[threadIdx.x >> 6] = e;
            __syncthreads();
            if (threadIdx.x == 0) {
                double tot = 0.0;
                for (int r = 0; r < (int)(blockDim.x >> 6); r++) tot += kc_red[r];
                if (!(tot * (1.0 + 1e-6) < (double)cd.slack)) atomicOr(&near_s, KV_NEAR_ARGMAX);
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) kc_n = 0;
        __syncthreads();
    };
    // the normalisation guard (max > 1e-9, detector.rs:165) under the common factor: the reference's
    // mode top lies in [(R_W - A_W) / (1 + cr), (R_W + A_W)(1 + cr)]
    auto kc_guard = [&](const float* raw, const float* SS, const float* V, double sf, double K) {
        int bits = 0;
        for (int m = 0; m < 2; m++) {
            int W = 0;
            for (int k = 1; k < 12; k++)
                if (!(raw[12 * m + k] < raw[12 * m + W])) W = k;
            const double R = raw[12 * m + W];
            const double A = V[12 * m + W] * sf * (1.0 + 2.0001 * KC_U) + kc_noise(R, SS[12 * m + W] * sf, K);
            const double cr = kc_crs, t = (double)1e-9f, lo = (R - A) / (1.0 + cr), hi = (R + A) * (1.0 + cr);
            if (!(lo > t) && !(hi <= t)) bits |= KV_NEAR_RANGE;
        }
        return bits;
    };
    // the heuristic's weighted chroma sums (detector.rs:344-368): i < 12 -> avg[i], 12 -> wsum
    auto avg_sum = [&](int64_t f0, int64_t n, int i) {
        if (!use_w && i == 12) return (float)n;
        float a = 0.0f;
#pragma unroll 4
        for (int64_t f = f0; f < f0 + n; f++) {
            const float wt = use_w ? w[f] : 1.0f;
            const float term = i == 12 ? wt : (use_w ? wt * cs[f * 12 + i] : cs[f * 12 + i]);
            a += (use_w && wt <= 0.0f) ? 0.0f : term;
        }
        return a;
    };
    auto write_out = [&](int key, float conf, float clarity, int used) {
        KeyOut r{};
        r.mode = key < 12 ? 0 : 1;
        r.tonic = key % 12;
        r.conf = conf;
        r.clarity = clarity;
        r.ok = 1;
        r.used_segments = used;
        r.weights_used = use_w;
        // the key is the argmax of the accumulated scores: a relative gap in (0, margin] could flip
        // it (an exact tie of winners is structural and stays exact, key_raw_near)
        r.near = P.near_check ? (near_s | ((conf > 0.0f && !(conf > KV_NEAR_CONF)) ? KV_NEAR_FINAL : 0)) : 0;
        out[trk] = r;
    };
    // full-slice detection: detect_key_weighted (+ the mode heuristic)
    auto detect_full = [&](int used_segments) {
        __syncthreads();
        const bool kc = cert && use_w;  // without weights nothing depends on the energies
        if (threadIdx.x < 24)
            acc[threadIdx.x] = kc ? wsd3(0, F, toff + threadIdx.x, &kc_ss[threadIdx.x], &kc_v[threadIdx.x])
                                  : wsd(0, F, toff + threadIdx.x);
        if (P.mh_on && threadIdx.x >= 24 && threadIdx.x < 37) acc[threadIdx.x] = avg_sum(0, F, threadIdx.x - 24);
        __syncthreads();
        if (kc) {  // the slice's within-mode argmaxes (its final key and confidence are structural)
            if (threadIdx.x == 0) {
                float raw[24];
                for (int k = 0; k < 24; k++) raw[k] = acc[k];
                const int b = kc_argmax(raw, kc_ss, kc_v, kc_sf(F), kc_K(F), 0, (int)F, kc_list, &kc_n) |
                              kc_guard(raw, kc_ss, kc_v, kc_sf(F), kc_K(F));
                if (b) atomicOr(&near_s, b);
            }
            kc_pair_pass();
        }
        if (threadIdx.x == 0) {
            float raw[24], sorted[24];
            int order[24];
            for (int k = 0; k < 24; k++) raw[k] = acc[k];
            if (P.near_check && key_raw_near(raw)) atomicOr(&near_s, KV_NEAR_ARGMAX);
            key_from_raw(raw, sorted, order);
            int key = order[0];
            float conf = sorted[0] > 0.0f ? sd_clampf((sorted[0] - sorted[1]) / sorted[0], 0.0f, 1.0f) : 0.0f;
            if (P.mh_on) mode_heuristic(sorted, order, acc + 24, acc[36], P, &key, &conf);
            write_out(key, conf, clarity_of(sorted), used_segments);
            put_dbg(sorted, order, key);
        }
    };
    if (P.ensemble) {  // detect_key_ensemble (detector.rs:881-978), src/lib.rs:1289-1299
        if (threadIdx.x < 48) acc[threadIdx.x] = wsd(0, F, threadIdx.x);
        __syncthreads();
        if (threadIdx.x == 0) {
            const float tot = P.kk_w + P.tp_w;
            const float kn = tot > 1e-9f ? P.kk_w / tot : 0.5f;
            const float tn = tot > 1e-9f ? P.tp_w / tot : 0.5f;
            float raw[24], sorted[24], sa[24], sb[24], comb[24];
            int order[24];
            for (int k = 0; k < 24; k++) raw[k] = acc[k];
            key_from_raw(raw, sorted, order);
            for (int i = 0; i < 24; i++) sa[order[i]] = sorted[i];
            for (int k = 0; k < 24; k++) raw[k] = acc[24 + k];
            key_from_raw(raw, sorted, order);
            for (int i = 0; i < 24; i++) sb[order[i]] = sorted[i];
            for (int k = 0; k < 24; k++) comb[k] = kn * sa[k] + tn * sb[k];
            float conf;
            from_table(comb, sorted, order, &conf);
            write_out(order[0], conf, clarity_of(sorted), 0);
            put_dbg(sorted, order, order[0]);
        }
        return;
    }
    // segment lists: multi-scale (detector.rs:546-719) or segment voting (src/lib.rs:1331-1436)
    int mode = 0;  // 0 full, 1 multi-scale, 2 segment voting
    if (P.ms_on && P.ms_n > 0) {
        int mn = P.ms_len[0];
        for (int i = 1; i < P.ms_n; i++) mn = min(mn, P.ms_len[i]);
        if (F >= mn) mode = 1;
    }
    if (mode == 0 && P.seg_voting && F >= P.seg_len) mode = 2;
    if (mode == 0) {
        detect_full(0);
        return;
    }
    if (threadIdx.x == 0) {
        int n = 0;
        for (int si = 0; si < (mode == 1 ? P.ms_n : 1); si++) {
            const int len = mode == 1 ? P.ms_len[si] : P.seg_len;
            const int hop = mode == 1 ? max(P.ms_hop, 1) : P.seg_hop;
            const float sw = mode == 1 ? (si < P.ms_nw ? P.ms_w[si] : 1.0f) : 1.0f;
            sc_len[si] = len;
            sc_w[si] = sw;
            sc_pfx[si] = n;
            if (!(len == 0 || len > F || sw <= 0.0f)) n += (int)((F - len) / hop) + 1;
        }
        sc_pfx[mode == 1 ? P.ms_n : 1] = n;
    }
    __syncthreads();
    const int nsc = mode == 1 ? P.ms_n : 1;
    const int nseg = sc_pfx[nsc];
    auto seg_of = [&](int sg, int64_t* start, int* len, float* sw) {
        int si = 0;
        while (si + 1 < nsc && sc_pfx[si + 1] <= sg) si++;
        const int hop = mode == 1 ? max(P.ms_hop, 1) : P.seg_hop;
        *start = (int64_t)(sg - sc_pfx[si]) * hop;
        *len = sc_len[si];
        *sw = sc_w[si];
    };
    float* S = seg_scratch + seg_off[it];
    const bool kc2 = cert && use_w && mode == 2;  // segment voting under the certificate
    for (int q = threadIdx.x; q < nseg * 24; q += blockDim.x) {
        int64_t st;
        int len;
        float sw;
        seg_of(q / 24, &st, &len, &sw);
        float* row = S + (size_t)(q / 24) * KV_ROW;
        if (kc2)
            row[q % 24] = wsd3(st, len, toff + q % 24, &row[64 + q % 24], &row[88 + q % 24]);
        else
            row[q % 24] = wsd(st, len, toff + q % 24);  // raw score
    }
    if (P.mh_on)
        for (int q = threadIdx.x; q < nseg * 13; q += blockDim.x) {
            int64_t st;
            int len;
            float sw;
            seg_of(q / 13, &st, &len, &sw);
            const int i = q % 13;
            S[(size_t)(q / 13) * KV_ROW + (i == 12 ? 51 : 52 + i)] = avg_sum(st, len, i);
        }
    __syncthreads();
    KV_T(3);
    for (int sg = threadIdx.x; sg < nseg; sg += blockDim.x) {
        float* row = S + (size_t)sg * KV_ROW;
        float raw[24], sorted[24];
        int order[24];
        for (int k = 0; k < 24; k++) raw[k] = row[k];
        if (P.near_check && key_raw_near(raw)) atomicOr(&near_s, KV_NEAR_ARGMAX);
        int64_t st;
        int len;
        float sw;
        seg_of(sg, &st, &len, &sw);
        if (kc2) {
            const int b = kc_argmax(raw, row + 64, row + 88, kc_sf(len), kc_K(len), st, len, kc_list, &kc_n) |
                          kc_guard(raw, row + 64, row + 88, kc_sf(len), kc_K(len));
            if (b) atomicOr(&near_s, b);
        }
        key_from_raw(raw, sorted, order);
        if (P.mh_on) {
            int key;
            float conf;
            mode_heuristic(sorted, order, row + 52, row[51], P, &key, &conf);
        }
        const float cl = clarity_of(sorted);
        float kc_dcl = 0.0f;
        if (kc2) {  // the clarity bound; the per-key score bounds replace the partial-sum totals
            float beta[24];
            int b = 0;
            kc_dcl = kc_up(kc_clarity(raw, row + 64, row + 88, kc_sf(len), kc_K(len), sorted, order, beta, &b));
            if (b) atomicOr(&near_s, b);
            for (int k = 0; k < 24; k++) row[64 + k] = beta[k];
            row[112] = kc_dcl;
        }
        for (int k = 0; k < 24; k++) {
            row[k] = sorted[k];
            row[24 + k] = (float)order[k];
        }
        row[48] = cl;
        const float gate = mode == 1 ? P.ms_min_cl : P.min_clarity;
        row[49] = cl >= gate ? 1.0f : 0.0f;
        if (P.near_check && sd_absf(cl - gate) <= sd_maxf(KV_NEAR_CLARITY, kc_dcl))
            atomicOr(&near_s, KV_NEAR_GATE);  // the segment gate (src/lib.rs:1380)
        row[50] = cl * sw;
    }
    __syncthreads();
    KV_T(4);
    if (kc2) kc_pair_pass();
    KV_T(5);
    if (threadIdx.x < 24) {
        const int key = threadIdx.x;
        float a = 0.0f;
        double pa = 0.0;  // the certificate: the sum of the fold's partial sums
        for (int sg = 0; sg < nseg; sg++) {
            const float* row = S + (size_t)sg * KV_ROW;
            if (row[49] == 0.0f) continue;
            for (int k = 0; k < 24; k++)
                if ((int)row[24 + k] == key) {
                    a += row[k] * row[50];
                    pa += (double)a;
                    break;
                }
        }
        acc[key] = a;
        if (kc2) kc_pa[key] = kc_up(pa);
    }
    if (threadIdx.x == 32) {
        int u = 0;
        float tw = 0.0f;
        for (int sg = 0; sg < nseg; sg++)
            if (S[(size_t)sg * KV_ROW + 49] != 0.0f) {
                u++;
                tw += S[(size_t)sg * KV_ROW + 50];
            }
        used_s = u;
        totw_s = tw;
    }
    __syncthreads();
    KV_T(6);
    const int used = used_s;
    const float totw = totw_s;
    if (used == 0 || (mode == 1 && totw <= 1e-12f)) {
        detect_full(used);
        return;
    }
    // the certificate's final key (src/lib.rs:1412-1424): acc_x = sum over the used segments of
    // RN(rs_x cl), so for the leader W and a competitor k the reference's difference moves by at most
    // sum (|rs_W - rs_k| dcl + (beta_W + beta_k)(cl + dcl))(1 + 4u) + 2.0001 u (rs_W + rs_k) cl (the
    // products) + 2.0001 u 1.01 (its partial sums): the segment clarity's error enters scaled by the
    // pair's score difference, not by the scores
    if (kc2) {
        if (threadIdx.x == 0) {
            float sorted[24], conf;
            int order[24];
            from_table(acc, sorted, order, &conf);
            kc_w = order[0];
        }
        __syncthreads();
        const int W = kc_w, k = threadIdx.x;
        if (k < 24 && k != W) {
            double D = 0.0;
            // a structural tie: in every used segment both keys hold a certified mode top (the same
            // RN(1 + 0.2f), bound 0), so the reference forms the same products for both and ties too
            bool tie = true;
            for (int sg = 0; sg < nseg; sg++) {
                const float* row = S + (size_t)sg * KV_ROW;
                if (row[49] == 0.0f) continue;
                double rW = 0.0, rK = 0.0;
                for (int j = 0; j < 24; j++) {
                    const int o = (int)row[24 + j];
                    rW = o == W ? (double)row[j] : rW;
                    rK = o == k ? (double)row[j] : rK;
                }
                const double cw = row[50], dc = row[112], bw = row[64 + W], bk = row[64 + k];
                tie = tie && rW == rK && bw == 0.0 && bk == 0.0;
                D += (__builtin_fabs(rW - rK) * dc + (bw + bk) * (cw + dc)) * (1.0 + 4.0001 * KC_U) +
                     2.0001 * KC_U * (rW + rK) * cw;
            }
            D += 2.0001 * KC_U * 1.01 * ((double)kc_pa[W] + (double)kc_pa[k]);
            if (!tie && !((double)acc[W] - (double)acc[k] > D + 1.01 * KC_U * (double)acc[W]))
                atomicOr(&near_s, KV_NEAR_FINAL);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float tab[24], sorted[24];
        int order[24];
        for (int k = 0; k < 24; k++) tab[k] = mode == 1 ? acc[k] / totw : acc[k];
        float conf;
        from_table(tab, sorted, order, &conf);
        write_out(order[0], conf, clarity_of(sorted), used);
        put_dbg(sorted, order, order[0]);
    }
    KV_T(7);
#ifdef SDSP_KV_PROF
    if (threadIdx.x == 0 && (blockIdx.x % 64) == 0)
        printf("kvprof blk %d nseg %d smooth %.1f weights %.1f segs %.1f segkey %.1f pair %.1f acc %.1f final %.1f us\n",
               (int)blockIdx.x, nseg, (kv_t[1] - kv_t[0]) * 0.01, (kv_t[2] - kv_t[1]) * 0.01, (kv_t[3] - kv_t[2]) * 0.01,
               (kv_t[4] - kv_t[3]) * 0.01, (kv_t[5] - kv_t[4]) * 0.01, (kv_t[6] - kv_t[5]) * 0.01, (kv_t[7] - kv_t[6]) * 0.01);
#endif
}

// ---- launchers ----
void launch_mask(float* mags, int stride, int B, const uint64_t* frame_pfx, const int* tracks, int n_items, int margin,
                 float power, hipStream_t st, bool smooth_only) {
    if (n_items == 0) return;
    const int bpt = (B + MASK_T - 1) / MASK_T;
    const size_t lds = (size_t)(2 * margin + 2 + margin + 1) * MASK_T * sizeof(float);
    const float p = sd_maxf(power, 1.0f);
    if (smooth_only) {
        if (margin == 0) return;  // smooth_spectrogram_time returns its input (extractor.rs:1250-1252)
        hipLaunchKernelGGL(k_mask<1>, dim3(n_items * bpt), dim3(MASK_T), lds, st, mags, stride, B, frame_pfx, tracks,
                           bpt, margin, power, 1);
        return;
    }
    if (margin == 12 && p == 2.0f) {
        hipLaunchKernelGGL((k_mask_r<12, 2>), dim3(n_items * bpt), dim3(MASK_T), 0, st, mags, stride, B, frame_pfx,
                           tracks, bpt, power);
        return;
    }
    if (p == 2.0f)
        hipLaunchKernelGGL(k_mask<2>, dim3(n_items * bpt), dim3(MASK_T), lds, st, mags, stride, B, frame_pfx, tracks,
                           bpt, margin, power, 0);
    else if (p == 1.0f)
        hipLaunchKernelGGL(k_mask<1>, dim3(n_items * bpt), dim3(MASK_T), lds, st, mags, stride, B, frame_pfx, tracks,
                           bpt, margin, power, 0);
    else
        hipLaunchKernelGGL(k_mask<0>, dim3(n_items * bpt), dim3(MASK_T), lds, st, mags, stride, B, frame_pfx, tracks,
                           bpt, margin, power, 0);
}
bool mask_band_ok(int margin, float power) { return margin == 12 && sd_maxf(power, 1.0f) == 2.0f; }
void launch_mask_band(float* mags, int stride, int B, const uint64_t* frame_pfx, const int* tracks, int n_items,
                      float power, int st_lo, int st_hi, float* part, uint64_t total, hipStream_t st, bool outside) {
    if (n_items == 0) return;
    const int bpt = (B + MASK_T - 1) / MASK_T;
    hipLaunchKernelGGL((k_mask_rp<12, 2>), dim3(n_items * bpt), dim3(MASK_T), 0, st, mags, stride, B, frame_pfx, tracks,
                       bpt, power, st_lo, st_hi, part, total, outside ? 1 : 0);
}
void launch_hpcp_band(const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                      int n_items, uint64_t n_tiles, const HpcpParams& P, const HarmEntry* harm, const float* part,
                      uint64_t total, float* chroma, float* energy, float* edel, hipStream_t st) {
    if (n_tiles == 0) return;
    const int nblk = (P.B + MASK_T - 1) / MASK_T;
    const dim3 grid((unsigned)n_tiles), block(HP_FRAMES);
#define SDSP_HB(K)                                                                                                   \
    hipLaunchKernelGGL(k_hpcp_band<K>, grid, block, 0, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, harm, part, \
                       nblk, total, chroma, energy, edel)
    if (P.K <= 8)
        SDSP_HB(8);
    else if (P.K <= 16)
        SDSP_HB(16);
    else if (P.K <= 24)
        SDSP_HB(24);
    else
        SDSP_HB(HP_KMAX);
#undef SDSP_HB
}
void launch_hpcp(const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                 int n_items, uint64_t n_tiles, const HpcpParams& P, const HarmEntry* harm, float* chroma,
                 float* energy, hipStream_t st) {
    if (n_tiles == 0) return;
    const dim3 grid((unsigned)n_tiles), block(HP_FRAMES);
    if (P.K <= 8)
        hipLaunchKernelGGL(k_hpcp<8>, grid, block, 0, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, harm, chroma,
                           energy);
    else if (P.K <= 16)
        hipLaunchKernelGGL(k_hpcp<16>, grid, block, 0, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, harm, chroma,
                           energy);
    else if (P.K <= 24)
        hipLaunchKernelGGL(k_hpcp<24>, grid, block, 0, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, harm, chroma,
                           energy);
    else
        hipLaunchKernelGGL(k_hpcp<HP_KMAX>, grid, block, 0, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, harm,
                           chroma, energy);
}
void launch_key_vote(const int* tracks, int n_items, const uint64_t* frame_pfx, float* chroma_raw,
                     const float* energy, float* chroma_s, float* weights, float* seg_scratch, const uint64_t* seg_off,
                     const float* tmpl, const KeyParams& P, KeyOut* out, hipStream_t st, KeyDbg* dbg,
                     const float* edel, float* wdel, bool alone) {
    if (n_items == 0) return;
    // a few tracks (the exact reruns of near-decision tracks, one-track calls) or a launch with
    // nothing beside it (the call's last sub-batch, `alone`): the latency of one track's workgroup
    // is the launch, and 1024 threads cut it (the segment scores in one round instead of three);
    // other sub-batches keep 256 threads, which fit beside the key-stream STFT
    // (a 1,024-thread workgroup fills its CU's 4 waves per SIMD: more tracks than CUs take two
    // rounds, so a lone launch of more tracks than CUs runs 512 threads, two workgroups per CU)
    int cus = 0;
    if (alone && n_items > KV_SMALL_ITEMS) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 0;
    }
    if (n_items <= KV_SMALL_ITEMS || (alone && n_items <= cus))
        hipLaunchKernelGGL(k_key_vote<1024>, dim3(n_items), dim3(1024), 0, st, tracks, n_items, frame_pfx, chroma_raw,
                           energy, chroma_s, weights, seg_scratch, seg_off, tmpl, P, out, dbg, edel, wdel);
    else if (alone)
        hipLaunchKernelGGL(k_key_vote<512>, dim3(n_items), dim3(512), 0, st, tracks, n_items, frame_pfx, chroma_raw,
                           energy, chroma_s, weights, seg_scratch, seg_off, tmpl, P, out, dbg, edel, wdel);
    else
        hipLaunchKernelGGL(k_key_vote<KV_THREADS>, dim3(n_items), dim3(KV_THREADS), 0, st, tracks, n_items, frame_pfx,
                           chroma_raw, energy, chroma_s, weights, seg_scratch, seg_off, tmpl, P, out, dbg, edel, wdel);
}

}  // namespace sdsp
