// HBM ceiling probe (MI355X_MICROARCH.md quotes 6.29 TB/s for a float4 copy): copy and read-only
// streams over 16 GiB buffers in several shapes, so the kernels' "fraction of achievable HBM" is
// measured against the best of them rather than one shape.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/hbm_ceiling.hip -o tools/micro/hbm_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); std::exit(1); } } while (0)

typedef float v4 __attribute__((ext_vector_type(4)));
// one float4 per thread, no loop (grid = n / 256 workgroups)
__global__ __launch_bounds__(256) void copy_flat(const v4* __restrict__ a, v4* __restrict__ b) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    b[i] = a[i];
}
// U float4 per thread in flight, contiguous per workgroup tile (tile = 256 U float4)
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_tile(const v4* __restrict__ a, v4* __restrict__ b) {
    const size_t base = blockIdx.x * (size_t)(256 * U) + threadIdx.x;
    v4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = NT ? __builtin_nontemporal_load(&a[base + 256 * u]) : a[base + 256 * u];
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (NT)
            __builtin_nontemporal_store(x[u], &b[base + 256 * u]);
        else
            b[base + 256 * u] = x[u];
    }
}
template <int U>
__global__ __launch_bounds__(256) void read_tile(const v4* __restrict__ a, float* __restrict__ out) {
    const size_t base = blockIdx.x * (size_t)(256 * U) + threadIdx.x;
    v4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = a[base + 256 * u];
    float s = 0.0f;
#pragma unroll
    for (int u = 0; u < U; u++) s += x[u].x + x[u].y + x[u].z + x[u].w;
    if (s == 12345.0f) out[0] = s;
}

int main() {
    const size_t bytes = (size_t)16 << 30;
    float *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n4 = bytes / 16;
    auto timed = [&](const char* name, double moved, auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; rep++) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0 && ms < best) best = ms;  // rep 0 warms the pages
        }
        std::printf("%-22s %.3f TB/s\n", name, moved / (best * 1e-3) / 1e12);
    };
    timed("copy flat (r+w)", 2.0 * bytes, [&] { hipLaunchKernelGGL(copy_flat, dim3(n4 / 256), dim3(256), 0, 0, (const v4*)a, (v4*)b); });
    timed("copy tile4 (r+w)", 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_tile<4, false>), dim3(n4 / 1024), dim3(256), 0, 0, (const v4*)a, (v4*)b); });
    timed("copy tile8 (r+w)", 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_tile<8, false>), dim3(n4 / 2048), dim3(256), 0, 0, (const v4*)a, (v4*)b); });
    timed("copy tile4 nt (r+w)", 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_tile<4, true>), dim3(n4 / 1024), dim3(256), 0, 0, (const v4*)a, (v4*)b); });
    timed("read tile4 (r)", 1.0 * bytes, [&] { hipLaunchKernelGGL((read_tile<4>), dim3(n4 / 1024), dim3(256), 0, 0, (const v4*)a, b); });
    timed("read tile8 (r)", 1.0 * bytes, [&] { hipLaunchKernelGGL((read_tile<8>), dim3(n4 / 2048), dim3(256), 0, 0, (const v4*)a, b); });
    return 0;
}
