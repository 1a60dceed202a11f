// Exhaustive GPU check (mantissa pairs) of D0, the mask quotient without D1's Newton step on the
// reciprocal: y = rcp(b) (the hardware reciprocal), q0 = a y, q = q0 + (a - b q0) y, against the
// correctly rounded a / b (-fhip-fp32-correctly-rounded-divide-sqrt).  Stops at the first chunk
// with mismatches.  hipcc --offload-arch=gfx950 -O3 -fhip-fp32-correctly-rounded-divide-sqrt -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float div_d0(float a, float b) {
    const float y = __builtin_amdgcn_rcpf(b);
    const float q0 = a * y;
    return __builtin_fmaf(__builtin_fmaf(-b, q0, a), y, q0);
}

__global__ void k_pairs(uint32_t a0, uint32_t na, unsigned long long* bad, uint32_t* ex) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // b mantissa index
    if (t >= (1u << 23)) return;
    const float b = __uint_as_float(0x3F800000u | t);
    unsigned long long n0 = 0;
    for (uint32_t i = 0; i < na; i++) {
        const float a = __uint_as_float(0x3F800000u | (a0 + i));
        if (__float_as_uint(div_d0(a, b)) != __float_as_uint(a / b)) {
            n0++;
            ex[0] = __float_as_uint(a);
            ex[1] = __float_as_uint(b);
        }
    }
    if (n0) atomicAdd(bad, n0);
}

int main() {
    unsigned long long* bad;
    uint32_t* ex;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&ex, 8);
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(ex, 0, 8);
    const dim3 grid((1u << 23) / 256), block(256);
    const uint32_t chunk = 1u << 13;
    unsigned long long hb = 0;
    uint32_t c = 0;
    for (; c < (1u << 23) / chunk; c++) {
        hipLaunchKernelGGL(k_pairs, grid, block, 0, 0, c * chunk, chunk, bad, ex);
        if (c % 32 == 31) {
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
            printf("a-chunks %u/%u: D0 %llu mismatches\n", c + 1, (1u << 23) / chunk, hb);
            fflush(stdout);
            if (hb) break;
        }
    }
    (void)hipDeviceSynchronize();
    uint32_t he[2];
    (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(he, ex, 8, hipMemcpyDeviceToHost);
    printf("D0: %llu mismatches in %u of 1024 a-chunks (e.g. a=0x%08x b=0x%08x)\n", hb, c + 1 > 1024 ? 1024 : c + 1, he[0], he[1]);
    return 0;
}
