// sdsp_device.hpp — shared device-side definitions for the gfx950 analyze_audio kernels.
//
// Numerics contract: every kernel performs the reference's f32 operations in the reference's
// order (sequential folds are kept sequential; see DESIGN.md "exactness"), builds with
// -ffp-contract=off, and evaluates transcendentals through include/sdsp_libm.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sdsp_libm.h"

namespace sdsp {

constexpr float EPS = 1e-10f;
constexpr int WAVE = 64;

// Raises the issuing wave's priority on its SIMD.  Used at the top of the short, latency-bound
// tempo-path kernels so that, running beside the key stream's VALU-heavy STFT waves, they are
// not starved of issue slots (their one-wave-per-track chains would otherwise stretch the tempo
// stream by far more than they cost the STFT).
#ifdef SDSP_NO_SETPRIO
#define SDSP_LATENCY_CRITICAL() ((void)0)
#else
#define SDSP_LATENCY_CRITICAL() __builtin_amdgcn_s_setprio(2)
#endif

struct cx {
    float re, im;
};
__device__ __forceinline__ cx cadd(cx a, cx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cx csub(cx a, cx b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cx cmul(cx w, cx z) { return {w.re * z.re - w.im * z.im, w.re * z.im + w.im * z.re}; }

// Out-of-line copies of the general transcendental paths, for unrolled loops that would
// otherwise inline them once per iteration (instruction-cache pressure).
__device__ __noinline__ inline float sd_powf_ool(float x, float y) { return sd_powf(x, y); }
__device__ __noinline__ inline float sd_logf_ool(float x) { return sd_logf(x); }

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2).  Renumber so
// that XCD x owns one contiguous range of logical blocks: kernels whose neighbouring blocks
// share input (overlapping STFT frames) then find it in their own L2.  Speed only; any
// placement is correct.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
    const uint32_t per = nb / 8, rem = nb % 8, x = b % 8, l = b / 8;
    return x < rem ? x * (per + 1) + l : rem * (per + 1) + (x - rem) * per + l;
}

// sd_maxf(a, b) for a second operand that is never NaN (a may be): identical result, without
// the NaN tests (sd_maxf(NaN, b) = b = (NaN > b ? NaN : b)).
__device__ __forceinline__ float max_bnn(float a, float b) { return a > b ? a : b; }

// max_bnn(v, 0) for a v that is never a signalling NaN (the spectrogram and everything computed
// from it are results of arithmetic, whose NaNs are quiet): the IEEE-mode v_max_f32 already returns
// 0 for a quiet NaN and +0 for -0, so the canonicalising max the compiler adds in front of a value
// it cannot see the origin of (a load, a phi) is left out
__device__ __forceinline__ float max0_quiet(float v) {
    float r;
    asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(v));
    return r;
}

// 4 waves per SIMD (at most 128 VGPRs): with the D1 quotient the compiler otherwise settles at
// 130 VGPRs and 3 waves, 2-3 % slower (profiles/r05_kernel_ab_mask_d1.txt)

// ---- wave / block reductions (order-free ops only: max, min, integer sums) ----
__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = sd_maxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Largest index i in [0, n) with pfx[i] <= key (pfx ascending, pfx[0] == 0): maps a flat
// work index onto its track for ragged batches.
__device__ __forceinline__ int find_track(const uint64_t* pfx, int n, uint64_t key) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (pfx[mid] <= key)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

}  // namespace sdsp
