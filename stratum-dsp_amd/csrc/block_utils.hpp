// block_utils.hpp — workgroup-level building blocks (ordered compaction, max, radix select,
// bitonic sort).  Only order-free reductions (max, integer counts) are done as trees; every
// f32 sum in the pipeline stays sequential in the reference's order.
#pragma once

#include "sdsp_device.hpp"

namespace sdsp {

// Block-wide max of one float per thread (NaN ignored like f32::max).  red: >= blockDim/64 floats.
__device__ inline float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < nw; i++) r = sd_maxf(r, red[i]);
    __syncthreads();
    return r;
}

// Sequential f32 sum p[0] + p[1] + ... + p[n-1] (the reference's fold order), returned to every
// thread.  The block stages SEQ_CH values at a time into LDS with coalesced loads; thread 0
// folds them in order.  buf: SEQ_CH floats of LDS.
constexpr int SEQ_CH = 2048;
__device__ inline float block_seq_sum(const float* p, int64_t n, float* buf) {
    __shared__ float res;
    float sum = 0.0f;
    for (int64_t c0 = 0; c0 < n; c0 += SEQ_CH) {
        const int64_t m = n - c0 < SEQ_CH ? n - c0 : SEQ_CH;
        __syncthreads();
        for (int i = threadIdx.x; i < m; i += blockDim.x) buf[i] = p[c0 + i];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int i = 0; i < m; i++) sum += buf[i];
    }
    if (threadIdx.x == 0) res = sum;
    __syncthreads();
    return res;
}

// Block-wide integer sum.
__device__ inline int block_sum_i(int v, int* red) {
    v = wave_sum_i(v);
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    int r = 0;
    for (int i = 0; i < nw; i++) r += red[i];
    __syncthreads();
    return r;
}

// Exclusive prefix of a 0/1 flag across the block, in thread order.  Returns this thread's
// slot; *total receives the number of set flags.  red: >= blockDim/64 + 1 ints.
__device__ inline int block_exclusive_flag(bool flag, int* red, int* total) {
    const unsigned long long b = __ballot(flag);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const unsigned long long lower = lane == 0 ? 0ull : (b & ((~0ull) >> (64 - lane)));
    const int in_wave = __popcll(lower);
    __syncthreads();
    if (lane == 0) red[w] = __popcll(b);
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < nw; i++) {
        if (i < w) base += red[i];
        tot += red[i];
    }
    __syncthreads();
    *total = tot;
    return base + in_wave;
}

// k-th smallest (0-based) of n non-negative, non-NaN floats in global memory, by 4x8-bit
// radix select on the IEEE bit pattern (monotone for x >= 0).  Exact and deterministic.
// hist: 256 ints of LDS; misc: >= 4 ints of LDS.
__device__ inline float block_select_kth(const float* x, int n, int k, int* hist, int* misc) {
    uint32_t prefix = 0, mask = 0;
    int kk = k;
    for (int pass = 3; pass >= 0; pass--) {
        const int shift = pass * 8;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const uint32_t u = sd_bits_f(x[i]);
            if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int acc = 0, d = 0;
            for (d = 0; d < 256; d++) {
                if (acc + hist[d] > kk) break;
                acc += hist[d];
            }
            misc[0] = d;
            misc[1] = kk - acc;
        }
        __syncthreads();
        prefix |= (uint32_t)misc[0] << shift;
        mask |= 255u << shift;
        kk = misc[1];
        __syncthreads();
    }
    return sd_from_bits_f(prefix);
}

// In-LDS bitonic sort of n (power of two) uint64 keys, ascending.
__device__ inline void block_bitonic_u64(uint64_t* keys, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int i = threadIdx.x; i < n / 2; i += blockDim.x) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool up = ((lo & size) == 0);
                const uint64_t a = keys[lo], b = keys[hi];
                if ((a > b) == up) {
                    keys[lo] = b;
                    keys[hi] = a;
                }
            }
        }
    }
    __syncthreads();
}

// Sort key helpers: non-negative float descending, ties by index ascending (== Rust's stable
// sort_by(|a, b| b.partial_cmp(a)) on NaN-free data).
__device__ __forceinline__ uint64_t key_desc_nonneg(float v, uint32_t idx) {
    return ((uint64_t)(~sd_bits_f(v)) << 32) | idx;
}
// Any finite float ascending (total order), ties by index.
__device__ __forceinline__ uint32_t ord_f(float v) {
    const uint32_t u = sd_bits_f(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint64_t key_asc(float v, uint32_t idx) { return ((uint64_t)ord_f(v) << 32) | idx; }
__device__ __forceinline__ uint64_t key_desc(float v, uint32_t idx) { return ((uint64_t)(~ord_f(v)) << 32) | idx; }

}  // namespace sdsp
