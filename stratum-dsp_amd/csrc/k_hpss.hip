// k_hpss.hip — hpss_decompose (reference src/features/onset/hpss.rs:71-281): ten rounds of a
// horizontal (time) and a vertical (frequency) median filter with soft re-partitioning of the
// original magnitudes, stopped per track once no element moves by 1e-6.  It feeds the HPSS onsets
// (src/lib.rs:222-236, hpss.rs:290-372) and the percussive tempogram fallback (src/lib.rs:587-683).
//
//   k_hpss_round    one round: frequency medians of P (LDS tile), time medians of H (registers),
//                   the re-partition and the change maximum, per 32-frame x 256-bin tile
//   k_hpss_conv     per-track convergence flags between rounds
//   k_hpss_rows     per-frame sum of squares (bin order) and max of the final P
//
// Medians: each thread slides a window along its row/column and keeps it sorted in registers.
// Inserting x into a sorted array b is c[j] = min(max(b[j-1], x), b[j]); deleting y (present) is
// d[j] = c[j] < y ? c[j] : c[j+1] (+inf pads the tail).  Both are 2 ops per slot on statically
// indexed registers.  The leaving value is deleted before the entering one is inserted, so the
// array never holds more than 2m + 1 <= W values.  The median of n values is s[n/2] for odd n and
// (s[n/2-1] + s[n/2]) * 0.5 for even n (the reference's windows shrink at the edges).
//
// Buffers ping-pong: round `it` reads H[it%2], P[it%2] (round 0: the spectrogram itself) and
// writes H[(it+1)%2], P[(it+1)%2]; the vertical filter reads a halo of P, so P cannot be updated
// in place.  Every buffer is addressed through per-track row offsets.
#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdsp {

namespace {

template <int W>
__device__ __forceinline__ void sw_insert(float (&a)[W], float x) {
    // a sorted ascending with +inf padding; the last slot (+inf while count < W) drops off
#pragma unroll
    for (int j = W - 1; j > 0; j--) a[j] = fminf(fmaxf(a[j - 1], x), a[j]);
    a[0] = fminf(x, a[0]);
}
template <int W>
__device__ __forceinline__ void sw_delete(float (&a)[W], float y) {
#pragma unroll
    for (int j = 0; j < W - 1; j++) a[j] = a[j] < y ? a[j] : a[j + 1];
    a[W - 1] = __builtin_inff();
}
// MM >= 0: the margin is the compile-time MM (the full-window median is register a[MM]);
// MM < 0: runtime m (a select chain).
template <int W, int MM>
__device__ __forceinline__ float sw_median(const float (&a)[W], int n, int m) {
    if constexpr (MM >= 0) {
        if (n == 2 * MM + 1) return a[MM];
    } else if (n == 2 * m + 1) {
        float v = a[0];
#pragma unroll
        for (int j = 0; j < W; j++)
            if (j == m) v = a[j];
        return v;
    }
    const int h = n / 2;
    float hi = 0.0f, lo = 0.0f;
#pragma unroll
    for (int j = 0; j < W; j++) {
        if (j == h) hi = a[j];
        if (j == h - 1) lo = a[j];
    }
    if (n & 1) return hi;
    return (lo + hi) * 0.5f;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// One round, fused.  A workgroup owns VM_ROWS frames x VM_COLS bins of one track:
//  1. the P tile with its +-m bin halo is staged in LDS; thread (row, segment) slides the
//     frequency median along VM_SEG bins of its row (results in registers);
//  2. thread b slides the time median of bin b down the tile's rows, reading H straight from
//     global memory (lanes are adjacent bins: coalesced rows; the +-m halo rows come from L2);
//  3. the frequency medians replace the tile centre and thread b re-partitions its column:
//     total = h + p; H', P' = orig * h/total, orig * p/total (or orig * 0.5 each when total <=
//     1e-10), and the round's change max(|H' - H|, |P' - P|) goes to the track's maximum.
// Per round the spectrogram-sized streams are H (+ halo), P, orig read and H', P' written.
constexpr int VM_ROWS = HPSS_VM_FRAMES, VM_SEG = 32, VM_COLS = HPSS_COLS, VM_MAXM = 16;
constexpr int VM_LD = VM_COLS + 2 * VM_MAXM + 1;
static_assert(VM_ROWS * (VM_COLS / VM_SEG) == 256 && VM_COLS == 256, "thread maps of k_hpss_round");
template <int W, int MM>
__global__ __launch_bounds__(256) void k_hpss_round(const float* __restrict__ orig, const uint64_t* __restrict__ o_row0,
                                                    const float* __restrict__ hin, const float* __restrict__ pin,
                                                    const uint64_t* __restrict__ in_row0, float* __restrict__ hout,
                                                    float* __restrict__ pout, const uint64_t* __restrict__ out_row0,
                                                    const uint64_t* __restrict__ fpfx, const uint64_t* __restrict__ tile_pfx,
                                                    const int* __restrict__ last_it, int it, int n_items, HpssParams P,
                                                    unsigned int* __restrict__ change) {
    __shared__ float tl[VM_ROWS][VM_LD];
    __shared__ float red[4];
    const uint64_t gb = blockIdx.x;
    const int k = find_track(tile_pfx, n_items, gb);
    if (last_it[k] < it) return;  // converged in an earlier round
    const int64_t F = (int64_t)(fpfx[k + 1] - fpfx[k]);
    const int ncb = (P.B + VM_COLS - 1) / VM_COLS;
    const int64_t lt = (int64_t)(gb - tile_pfx[k]);
    const int64_t r0 = (lt / ncb) * VM_ROWS;
    const int c0 = (int)(lt % ncb) * VM_COLS;
    const int m = MM >= 0 ? MM : P.m, B = P.B;
    const uint64_t stride = (uint64_t)P.stride;
    const uint64_t ir = in_row0[k], orr = out_row0[k], oo = o_row0[k];
    // 1. stage P rows r0.., bins c0-m .. c0+VM_COLS+m; frequency medians
    const int cols = VM_COLS + 2 * m;
    for (int e = threadIdx.x; e < VM_ROWS * cols; e += 256) {
        const int r = e / cols, c = e % cols;
        const int64_t t = r0 + r;
        const int b = c0 - m + c;
        float v = 0.0f;
        if (t < F && b >= 0 && b < B) v = pin[(ir + (uint64_t)t) * stride + b];
        tl[r][c] = v;
    }
    __syncthreads();
    const int r = threadIdx.x % VM_ROWS, sg = threadIdx.x / VM_ROWS;
    const int bs = c0 + sg * VM_SEG;
    float pf[VM_SEG];
    {
        float a[W];
#pragma unroll
        for (int j = 0; j < W; j++) a[j] = __builtin_inff();
        const int w0 = bs >= m ? bs - m : 0, w1 = bs + m + 1 < B ? bs + m + 1 : B;
        for (int b = w0; b < w1; b++) sw_insert<W>(a, tl[r][b - c0 + m]);
        int n = w1 - w0;
#pragma unroll
        for (int j = 0; j < VM_SEG; j++) {
            const int b = bs + j;
            pf[j] = b < B ? sw_median<W, MM>(a, n, m) : 0.0f;
            if (j + 1 == VM_SEG || b + 1 >= B) continue;  // no further median in this segment
            const int bin = b + m + 1, bout = b - m;
            if (bout >= 0) {
                sw_delete<W>(a, tl[r][bout - c0 + m]);
                n--;
            }
            if (bin < B) {
                sw_insert<W>(a, tl[r][bin - c0 + m]);
                n++;
            }
        }
    }
    // 2. time medians of bin b over the tile's rows
    const int b = c0 + (int)threadIdx.x;
    const bool col = b < B;
    float hf[VM_ROWS];
    if (col) {
        const float* src = hin + ir * stride + b;
        float a[W];
#pragma unroll
        for (int j = 0; j < W; j++) a[j] = __builtin_inff();
        const int64_t w0 = r0 >= m ? r0 - m : 0, w1 = r0 + m + 1 < F ? r0 + m + 1 : F;
        for (int64_t t = w0; t < w1; t++) sw_insert<W>(a, src[(uint64_t)t * stride]);
        int n = (int)(w1 - w0);
#pragma unroll
        for (int j = 0; j < VM_ROWS; j++) {
            const int64_t t = r0 + j;
            hf[j] = 0.0f;
            if (t < F) {
                hf[j] = sw_median<W, MM>(a, n, m);
                const int64_t tin = t + m + 1, tout = t - m;
                if (tout >= 0) {
                    sw_delete<W>(a, src[(uint64_t)tout * stride]);
                    n--;
                }
                if (tin < F) {
                    sw_insert<W>(a, src[(uint64_t)tin * stride]);
                    n++;
                }
            }
        }
    }
    // 3. re-partition, one column per thread
    __syncthreads();
#pragma unroll
    for (int j = 0; j < VM_SEG; j++) tl[r][sg * VM_SEG + j + m] = pf[j];
    __syncthreads();
    float mx = 0.0f;
    if (col) {
#pragma unroll
        for (int j = 0; j < VM_ROWS; j++) {
            const int64_t t = r0 + j;
            if (t >= F) break;
            const float x = orig[(oo + (uint64_t)t) * stride + b];
            const float h = hf[j];
            const float p = tl[j][threadIdx.x + m];
            const float total = h + p;
            float hn, pn;
            if (total > 1e-10f) {
                hn = x * (h / total);
                pn = x * (p / total);
            } else {
                hn = x * 0.5f;
                pn = x * 0.5f;
            }
            const uint64_t ou = (orr + (uint64_t)t) * stride + b;
            hout[ou] = hn;
            pout[ou] = pn;
            if (it > 0) {
                const uint64_t io = (ir + (uint64_t)t) * stride + b;
                mx = sd_maxf(sd_maxf(mx, sd_absf(hn - hin[io])), sd_absf(pn - pin[io]));
            }
        }
    }
    if (it > 0) {
        mx = block_max(mx, red);
        if (threadIdx.x == 0 && mx > 0.0f) atomicMax(&change[k], sd_bits_f(mx));
    }
}

// Round `it` done: a track whose largest change is < 1e-6 (it > 0) stops (hpss.rs:160-170).
__global__ void k_hpss_conv(int n_items, int it, unsigned int* __restrict__ change, int* __restrict__ last_it) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_items) return;
    if (last_it[k] >= it && it > 0 && sd_from_bits_f(change[k]) < 1e-6f) last_it[k] = it;
    change[k] = 0;
}

// Final P -> P0 for tracks that stopped after an even round (their result sits in P[1]).
__global__ __launch_bounds__(256) void k_hpss_final(float* __restrict__ p0, const float* __restrict__ p1,
                                                    const uint64_t* __restrict__ row0, const uint64_t* __restrict__ fpfx,
                                                    const int* __restrict__ last_it, int n_items, int stride, int B) {
    const int k = blockIdx.y;
    if (k >= n_items || (last_it[k] & 1)) return;  // odd round -> written to P[0]
    const uint64_t F = fpfx[k + 1] - fpfx[k];
    const uint64_t n = F * (uint64_t)stride;
    const uint64_t base = row0[k] * (uint64_t)stride;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        if ((int)(i % (uint64_t)stride) < B) p0[base + i] = p1[base + i];
}

// Per-frame sum of squares in bin order (hpss.rs:305-309) and the frame maximum (the spectral-flux
// normalisation of a tempogram pass over P), one thread per frame; bins staged through LDS.
constexpr int RW_T = 256, RW_CW = 16;
__global__ __launch_bounds__(RW_T) void k_hpss_rows(const float* __restrict__ p, const uint64_t* __restrict__ row0,
                                                    const uint64_t* __restrict__ fpfx,
                                                    const uint64_t* __restrict__ tile_pfx, int n_items, int stride,
                                                    int B, float* __restrict__ energy, float* __restrict__ fmax) {
    __shared__ float tile[RW_T][RW_CW + 1];
    const uint64_t gb = blockIdx.x;
    const int k = find_track(tile_pfx, n_items, gb);
    const int64_t F = (int64_t)(fpfx[k + 1] - fpfx[k]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[k]) * RW_T;
    const int i = threadIdx.x;
    const int sub = i / RW_CW, jj = i % RW_CW;
    const int64_t rows = F - f0 < RW_T ? F - f0 : RW_T;
    const float* base = p + (row0[k] + (uint64_t)f0) * (uint64_t)stride;
    float e = 0.0f, mx = 0.0f;
    for (int c0 = 0; c0 < B; c0 += RW_CW) {
        __syncthreads();
        for (int u = 0; u < RW_CW; u++) {
            const int rr = sub + u * (RW_T / RW_CW);
            tile[rr][jj] = (rr < rows && c0 + jj < B) ? base[(uint64_t)rr * stride + c0 + jj] : 0.0f;
        }
        __syncthreads();
        if (i < rows) {
            const int cw = B - c0 < RW_CW ? B - c0 : RW_CW;
            for (int j = 0; j < cw; j++) {
                const float v = tile[i][j];
                e += v * v;
                mx = sd_maxf(mx, v);
            }
        }
    }
    if (i < rows) {
        energy[fpfx[k] + (uint64_t)(f0 + i)] = e;
        fmax[fpfx[k] + (uint64_t)(f0 + i)] = mx;
    }
}

// ---- launcher: the whole decomposition ----
template <int W, int MM>
static void hpss_rounds(const HpssLaunch& L, hipStream_t st) {
    const HpssParams& P = L.P;
    for (int it = 0; it < 10; it++) {
        const float* hin = it == 0 ? L.orig : L.h[it % 2];
        const float* pin = it == 0 ? L.orig : L.p[it % 2];
        const uint64_t* irow = it == 0 ? L.orig_row0 : L.row0;
        float* hout = L.h[(it + 1) % 2];
        float* pout = L.p[(it + 1) % 2];
        hipLaunchKernelGGL((k_hpss_round<W, MM>), dim3((unsigned)L.n_vtiles), dim3(256), 0, st, L.orig, L.orig_row0, hin,
                           pin, irow, hout, pout, L.row0, L.fpfx, L.vtile_pfx, L.last_it, it, L.n_items, P, L.change);
        hipLaunchKernelGGL(k_hpss_conv, dim3((L.n_items + 255) / 256), dim3(256), 0, st, L.n_items, it, L.change,
                           L.last_it);
    }
    // round 9 writes P[0]; a track that stopped after round it sits in P[(it + 1) % 2]
    hipLaunchKernelGGL(k_hpss_final, dim3(64, L.n_items), dim3(256), 0, st, L.p[0], L.p[1], L.row0, L.fpfx, L.last_it,
                       L.n_items, P.stride, P.B);
}

void launch_hpss(const HpssLaunch& L, hipStream_t st) {
    if (L.n_items == 0) return;
    (void)hipMemsetAsync(L.change, 0, (size_t)L.n_items * sizeof(unsigned int), st);
    if (L.P.m == 10)  // the default margin
        hpss_rounds<21, 10>(L, st);
    else if (L.P.m <= 4)
        hpss_rounds<9, -1>(L, st);
    else
        hpss_rounds<2 * VM_MAXM + 1, -1>(L, st);
}

void launch_hpss_rows(const float* p, const uint64_t* row0, const uint64_t* fpfx, const uint64_t* tile_pfx,
                      uint64_t n_tiles, int n_items, int stride, int B, float* energy, float* fmax, hipStream_t st) {
    if (n_tiles == 0) return;
    hipLaunchKernelGGL(k_hpss_rows, dim3((unsigned)n_tiles), dim3(RW_T), 0, st, p, row0, fpfx, tile_pfx, n_items,
                       stride, B, energy, fmax);
}

}  // namespace sdsp
