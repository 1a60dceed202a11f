// Token-ring latency between workgroups on different CUs (gfx950), for a cross-workgroup
// hand-off of per-frame partial sums (the key path's energy fold).  G one-wave
// workgroups pass a 64-float vector round a ring R times; each hop: poll the predecessor's flag,
// read its vector, add one, write own vector, wait for the stores, publish the flag.  Buffers are
// either uncached device memory (hipDeviceMallocUncached, plain volatile accesses) or ordinary
// device memory with agent-scope release / acquire atomics.  Every spin is bounded: a timeout sets
// err and the kernel ends.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/uc_chain.hip -o tools/micro/uc_chain && ./uc_chain
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

template <bool UC>
__global__ __launch_bounds__(64) void ring(unsigned* flag, float* data, int G, int R, unsigned* err) {
    const int g = blockIdx.x, lane = threadIdx.x;
    const int prev = (g + G - 1) % G;
    for (int r = 1; r <= R; r++) {
        const unsigned need = g == 0 ? (unsigned)(r - 1) : (unsigned)r;  // group 0 waits for the ring's last hop
        if (!(g == 0 && r == 1)) {
            long spins = 0;
            while (true) {
                unsigned f;
                if (UC)
                    f = *(volatile unsigned*)&flag[prev];
                else
                    f = __hip_atomic_load(&flag[prev], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (f >= need) break;
                if (++spins > (1l << 22)) {
                    if (lane == 0) atomicOr(err, 1u);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        float v;
        if (UC)
            v = ((volatile float*)data)[prev * 64 + lane];
        else
            v = data[prev * 64 + lane];
        v = (g == 0 ? (float)(r * 1000) : v + 1.0f);
        if (UC) {
            ((volatile float*)data)[g * 64 + lane] = v;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) *(volatile unsigned*)&flag[g] = (unsigned)r;
        } else {
            data[g * 64 + lane] = v;
            if (lane == 0) __hip_atomic_store(&flag[g], (unsigned)r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int main() {
    const int G = 65, R = 2000;
    for (int uc = 1; uc >= 0; uc--) {
        unsigned *flag, *err;
        float* data;
        if (uc) {
            hipExtMallocWithFlags((void**)&flag, G * 4, hipDeviceMallocUncached);
            hipExtMallocWithFlags((void**)&data, G * 64 * 4, hipDeviceMallocUncached);
        } else {
            hipMalloc(&flag, G * 4);
            hipMalloc(&data, G * 64 * 4);
        }
        hipMalloc(&err, 4);
        hipMemset(flag, 0, G * 4);
        hipMemset(data, 0, G * 64 * 4);
        hipMemset(err, 0, 4);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        if (uc)
            hipLaunchKernelGGL(ring<true>, dim3(G), dim3(64), 0, 0, flag, data, G, R, err);
        else
            hipLaunchKernelGGL(ring<false>, dim3(G), dim3(64), 0, 0, flag, data, G, R, err);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        unsigned e = 0;
        float last = 0;
        hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
        hipMemcpy(&last, data + (G - 1) * 64, 4, hipMemcpyDeviceToHost);
        std::printf("%s: %.3f ms for %d hops -> %.3f us per hop; err %u; last %.0f (want %d)\n",
                    uc ? "uncached volatile" : "agent acq/rel", ms, G * R, 1000.0 * ms / (G * R), e, last,
                    R * 1000 + G - 1);
        hipFree(flag);
        hipFree(data);
        hipFree(err);
    }
    return 0;
}
