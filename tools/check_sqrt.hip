// Exhaustive GPU check: sqrt_cr (k_stft.hip) == sqrtf (correctly rounded) for every f32 bit
// pattern in [0, +inf].  hipcc --offload-arch=gfx950 -O3 -fhip-fp32-correctly-rounded-divide-sqrt
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ __forceinline__ float sqrt_cr(float x) {
    if (__builtin_expect(x >= 0x1p-96f && x < __builtin_huge_valf(), 1)) {
        float s = __builtin_amdgcn_sqrtf(x);
        const float sm = __uint_as_float(__float_as_uint(s) - 1u);
        const float sp = __uint_as_float(__float_as_uint(s) + 1u);
        const float rm = __builtin_fmaf(-sm, s, x);
        const float rp = __builtin_fmaf(-sp, s, x);
        s = rm <= 0.0f ? sm : s;
        s = rp > 0.0f ? sp : s;
        return s;
    }
    return __builtin_sqrtf(x);
}
__global__ void k(unsigned long long* bad, unsigned* first) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > 0x7f800000ull) return;
    const float x = __uint_as_float((uint32_t)i);
    const float a = sqrt_cr(x), b = __builtin_sqrtf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) { atomicAdd(bad, 1ull); atomicMin(first, (unsigned)i); }
}
int main() {
    unsigned long long* bad; unsigned* first;
    hipMalloc(&bad, 8); hipMalloc(&first, 4);
    hipMemset(bad, 0, 8); unsigned big = 0xffffffffu; hipMemcpy(first, &big, 4, hipMemcpyHostToDevice);
    const uint64_t n = 0x7f800001ull;
    hipLaunchKernelGGL(k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, bad, first);
    unsigned long long hb; unsigned hf;
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    printf("sqrt_cr vs sqrtf over all non-negative f32: %llu mismatches (first 0x%08x)\n", hb, hf);
    return hb != 0;
}
