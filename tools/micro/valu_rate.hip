// VALU issue-rate probe (gfx950): wave-instructions per SIMD per ns for v_fma_f32, v_pk_fma_f32,
// v_add_f32, v_pk_add_f32 and dependent-chain variants, at 1..8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip ; run: ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096

template <int KIND>
__global__ void k(float* out, float seed) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = seed * 0.5f, c = seed * 0.25f;
    for (int i = 0; i < ITERS; i++) {
        if constexpr (KIND == 0) {  // 8 independent v_fma_f32
            asm volatile(
                "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
                "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(b), "v"(c));
        } else if constexpr (KIND == 1) {  // 4 independent v_pk_fma_f32 on register pairs = 8 lanes of work
            asm volatile(
                "v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5\n"
                "v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5\n"
                : "+v"(*(double*)&a0), "+v"(*(double*)&a2), "+v"(*(double*)&a4), "+v"(*(double*)&a6)
                : "v"(*(double*)&b), "v"(*(double*)&b));
        } else if constexpr (KIND == 2) {  // 8 dependent v_fma_f32 (one chain)
            asm volatile(
                "v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n"
                "v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n"
                : "+v"(a0)
                : "v"(b), "v"(c));
        } else if constexpr (KIND == 3) {  // 8 independent v_add_f32
            asm volatile(
                "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(b));
        } else if constexpr (KIND == 4) {  // 8 independent v_pk_add_f32
            asm volatile(
                "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                : "+v"(*(double*)&a0), "+v"(*(double*)&a2), "+v"(*(double*)&a4), "+v"(*(double*)&a6)
                : "v"(*(double*)&b));
        } else if constexpr (KIND == 5) {  // 8 independent v_mul_f32
            asm volatile(
                "v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n v_mul_f32 %3, %3, %8\n"
                "v_mul_f32 %4, %4, %8\n v_mul_f32 %5, %5, %8\n v_mul_f32 %6, %6, %8\n v_mul_f32 %7, %7, %8\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(b));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int KIND>
void run(const char* name, float* d) {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    for (int wps : {1, 2, 4, 8}) {
        const int block = 256;                  // 4 waves = one per SIMD
        const int grid = cus * wps;             // wps workgroups per CU -> wps waves per SIMD
        hipLaunchKernelGGL(k<KIND>, dim3(grid), dim3(block), 0, 0, d, 1.0f);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<KIND>, dim3(grid), dim3(block), 0, 0, d, 1.0f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double instr_per_simd = 5.0 * wps * (double)ITERS * 8;  // wave-instructions per SIMD
        printf("%-28s waves/SIMD %d: %.3f ms, %.3f ns per wave-instruction per SIMD (%.2f cycles at 2.4 GHz)\n", name,
               wps, ms, ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
    }
}

int main() {
    float* d;
    hipMalloc(&d, 256 * 1024 * 16 * sizeof(float));
    run<0>("v_fma_f32 x8 indep", d);
    run<1>("v_pk_fma_f32 x8 (4 pairs)", d);
    run<2>("v_fma_f32 x8 dependent", d);
    run<3>("v_add_f32 x8 indep", d);
    run<4>("v_pk_add_f32 x8 (4 pairs)", d);
    run<5>("v_mul_f32 x8 indep", d);
    return 0;
}
