// Read-pattern probe for k_mask_rp (gfx950): one wave per (track, 64-bin block) streams the
// track's frames in blocks of 26 rows, one float per lane per row, as the mask does; the bins
// are laid out either row-major (frame rows of 4160 floats: each wave-row is a 256-byte segment
// 16 KB from the next) or block-major ([block][frame][64]: a wave's 26 rows are 6.6 KB
// contiguous).  Same bytes, same loads in flight; the values are summed so nothing is elided.
// Build: hipcc --offload-arch=gfx950 -O3 -o mask_layout mask_layout.hip ; run: ./mask_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int NB = 65, ROW = NB * 64, R = 26;  // rows padded to whole blocks: both layouts span T F ROW floats

template <bool BLOCK_MAJOR>
__global__ __launch_bounds__(64) void k_read(const float* __restrict__ x, int F, float* __restrict__ out) {
    const int trk = blockIdx.x / NB, g = blockIdx.x % NB, lane = threadIdx.x;
    const float* base = BLOCK_MAJOR ? x + ((uint64_t)trk * NB + g) * (uint64_t)F * 64 + lane
                                    : x + (uint64_t)trk * F * ROW + g * 64 + lane;
    const uint64_t step = BLOCK_MAJOR ? 64 : ROW;
    float acc = 0.0f, xv[R];
#pragma unroll
    for (int u = 0; u < R; u++) xv[u] = __builtin_nontemporal_load(base + u * step);
    for (int b = 0; b < F; b += R) {
        float s = 0.0f;
#pragma unroll
        for (int u = 0; u < R; u++) s += xv[u] * xv[u];
        acc += s;
        if (b + 2 * R <= F) {
#pragma unroll
            for (int u = 0; u < R; u++) xv[u] = __builtin_nontemporal_load(base + (uint64_t)(b + R + u) * step);
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

int main() {
    const int T = 96, F = 15496;  // 96 tracks of 3 min at hop 512
    const uint64_t n = (uint64_t)T * F * ROW;
    float *x, *out;
    hipMalloc(&x, n * 4);
    hipMalloc(&out, (size_t)T * NB * 64 * 4);
    hipMemset(x, 0, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        for (int bm = 0; bm < 2; bm++) {
            hipEventRecord(e0);
            if (bm) hipLaunchKernelGGL(k_read<true>, dim3(T * NB), dim3(64), 0, 0, x, F, out);
            else hipLaunchKernelGGL(k_read<false>, dim3(T * NB), dim3(64), 0, 0, x, F, out);
            hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess) {
                printf("launch failed\n");
                return 1;
            }
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (double)T * NB * 64 * 4 * (double)((F / R) * R);
            printf("%s rep %d: %.3f ms  %.2f TB/s\n", bm ? "block-major" : "row-major  ", rep, ms, bytes / ms / 1e9);
        }
    }
    return 0;
}
