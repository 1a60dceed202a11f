// Exhaustive GPU check of cheaper correctly rounded f32 sqrt sequences for the STFT magnitudes:
// each variant against sqrtf (correctly rounded under -fhip-fp32-correctly-rounded-divide-sqrt)
// for x = +0 and every f32 in [2^-96, +inf] (the range k_stft_slide8's fast path serves; other
// inputs go to the redo list).
//   hipcc --offload-arch=gfx950 -O3 -fhip-fp32-correctly-rounded-divide-sqrt -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

// A: Markstein's rsqrt step: y ~ 1/sqrt(x), s0 = x y, h = y / 2, r = x - s0^2 (exact, FMA),
//    s = s0 + r h.  x = +0: y from max(x, 2^-126) is finite, so s0 = 0 and s = +0.
__device__ __forceinline__ float sqrt_a(float x) {
    const float y = __builtin_amdgcn_rsqf(__builtin_fmaxf(x, 0x1p-126f));
    const float s0 = x * y, h = 0.5f * y;
    const float r = __builtin_fmaf(-s0, s0, x);
    return __builtin_fmaf(r, h, s0);
}
// B: the same step from v_sqrt's result: s0 = sqrt~(x), r = x - s0^2, s = s0 + r (0.5 / s0)
__device__ __forceinline__ float sqrt_b(float x) {
    const float s0 = __builtin_amdgcn_sqrtf(x);
    const float h = 0.5f * __builtin_amdgcn_rcpf(__builtin_fmaxf(s0, 0x1p-63f));
    const float r = __builtin_fmaf(-s0, s0, x);
    return __builtin_fmaf(r, h, s0);
}
// C: A with the half folded into the residual: s = s0 + (0.5 r) y
__device__ __forceinline__ float sqrt_c(float x) {
    const float y = __builtin_amdgcn_rsqf(__builtin_fmaxf(x, 0x1p-126f));
    const float s0 = x * y;
    const float r = __builtin_fmaf(-s0, s0, x);
    return __builtin_fmaf(0.5f * r, y, s0);
}

__global__ void k(unsigned long long* bad, unsigned* first) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > 0x7f800000ull) return;
    const uint32_t u = (uint32_t)i;
    const float x = __uint_as_float(u);
    if (u != 0 && u < 0x0F800000u) {  // (0, 2^-96): A and C reported separately over this range
        const uint32_t ref = __float_as_uint(__builtin_sqrtf(x));
        if (__float_as_uint(sqrt_a(x)) != ref) atomicAdd(&bad[3], 1ull);
        if (__float_as_uint(sqrt_c(x)) != ref) atomicAdd(&bad[4], 1ull);
        return;
    }
    const uint32_t ref = __float_as_uint(__builtin_sqrtf(x));
    const uint32_t v[3] = {__float_as_uint(sqrt_a(x)), __float_as_uint(sqrt_b(x)), __float_as_uint(sqrt_c(x))};
    for (int j = 0; j < 3; j++)
        if (v[j] != ref) {
            atomicAdd(&bad[j], 1ull);
            atomicMin(&first[j], u);
        }
}
int main() {
    unsigned long long* bad;
    unsigned* first;
    hipMalloc(&bad, 5 * 8);
    hipMalloc(&first, 3 * 4);
    hipMemset(bad, 0, 5 * 8);
    hipMemset(first, 0xff, 3 * 4);
    const uint64_t n = 0x7f800001ull;
    hipLaunchKernelGGL(k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, bad, first);
    unsigned long long hb[5];
    unsigned hf[3];
    hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost);
    hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost);
    const char* nm[3] = {"A rsq+Markstein", "B sqrt+rcp step", "C rsq, half in residual"};
    for (int j = 0; j < 3; j++) printf("%-24s %llu mismatches (first 0x%08x)\n", nm[j], hb[j], hf[j]);
    printf("(0, 2^-96): A %llu mismatches, C %llu mismatches\n", hb[3], hb[4]);
    return 0;
}
