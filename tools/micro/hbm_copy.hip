// HBM ceiling probe: read+write streaming bandwidth of (a) a coalesced float4 copy and (b) the
// mask kernel's access pattern (a wave per 64-column group walking rows `stride` floats apart,
// 26 rows loaded then written), and (c) a read-only coalesced reduction.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/hbm_copy.hip -o tools/micro/hbm_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); std::exit(1); } } while (0)

typedef float v4 __attribute__((ext_vector_type(4)));
__global__ void copy4(const v4* __restrict__ a, v4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&a[i]), &b[i]);
}
__global__ void read4(const v4* __restrict__ a, float* __restrict__ out, size_t n) {
    float s = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const v4 v = __builtin_nontemporal_load(&a[i]);
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.0f) out[0] = s;
}
// columns of `cols` floats, rows `stride` apart, `rows` rows per column group; a 64-lane wave per
// 64-column group walks its rows in blocks of 26 (loads, then stores in place)
__global__ __launch_bounds__(64) void colwalk(float* __restrict__ m, int stride, int cols, int rows, int groups_per_track) {
    const int trk = blockIdx.x / groups_per_track, g = blockIdx.x % groups_per_track;
    const int b = g * 64 + threadIdx.x;
    if (b >= cols) return;
    float* col = m + (size_t)trk * rows * stride + b;
    for (int base = 0; base + 26 <= rows; base += 26) {
        float x[26];
#pragma unroll
        for (int u = 0; u < 26; u++) x[u] = __builtin_nontemporal_load(&col[(size_t)(base + u) * stride]);
#pragma unroll
        for (int u = 0; u < 26; u++) __builtin_nontemporal_store(x[u] * 1.0001f, &col[(size_t)(base + u) * stride]);
    }
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
    float ms;
    const size_t n4 = bytes / 16;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(copy4, dim3(256 * 64), dim3(256), 0, 0, (const v4*)a, (v4*)b, n4);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("copy4     %.2f TB/s (r+w)\n", 2.0 * bytes / (ms * 1e-3) / 1e12);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(read4, dim3(256 * 64), dim3(256), 0, 0, (const v4*)a, b, n4);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("read4     %.2f TB/s (r)\n", 1.0 * bytes / (ms * 1e-3) / 1e12);
        // the mask's shape: 4097 columns, stride 4104, 15,522 rows per track
        const int stride = 4104, cols = 4097, rows = 15522, gpt = (cols + 63) / 64;
        const int tracks = (int)(bytes / ((size_t)rows * stride * 4));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(colwalk, dim3(tracks * gpt), dim3(64), 0, 0, a, stride, cols, rows, gpt);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double moved = 2.0 * tracks * (double)(rows / 26 * 26) * cols * 4;
        std::printf("colwalk   %.2f TB/s (r+w, %d tracks)\n", moved / (ms * 1e-3) / 1e12, tracks);
    }
    return 0;
}
