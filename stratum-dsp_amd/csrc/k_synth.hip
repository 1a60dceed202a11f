// k_synth.hip — seeded synthetic tracks generated in HBM (SURVEY.md §8d recipe), so the
// throughput benchmark never pays PCIe for its inputs.  Per track: kick on every beat
// (60/120/180 Hz at 0.6/0.3/0.1, e^-10t, 100 ms: reference scripts/generate_fixtures.py:41-61),
// a noise hat half-way between beats (30 ms, e^-60t, 0.15), a sustained tonic triad and a
// diatonic 8th-note line (3 harmonics each, 0.2), then peak-normalised to 0.9 by the
// runtime (k_peak_abs + a scale pass).
#include "kernels.hpp"

namespace sdsp {

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ float tone3(float f, double t) {
    float s = 0.0f;
    for (int h = 1; h <= 3; h++) {
        double ph = f * h * t;
        ph -= (double)(int64_t)ph;
        s += __sinf((float)(6.283185307179586 * ph)) / (float)h;
    }
    return s;
}

__global__ __launch_bounds__(256) void k_synth(float* __restrict__ out, uint64_t len, uint32_t sr,
                                               const float* __restrict__ bpm_arr, const int* __restrict__ key_arr,
                                               uint64_t seed0) {
    const int trk = blockIdx.y;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const float bpm = bpm_arr[trk];
    const int key = key_arr[trk];
    const int mode = key / 12, tonic = key % 12;
    const uint64_t seed = 0x5EED0000ull + seed0 + (uint64_t)trk;
    const double t = (double)i / (double)sr;
    const double beat = 60.0 / (double)bpm;
    const double bi = (double)(int64_t)(t / beat);
    float x = 0.0f;
    const double tb = t - bi * beat;
    if (tb < 0.1) {
        const float e = __expf(-(float)tb * 10.0f);
        x += (0.6f * __sinf((float)(6.283185307179586 * 60.0 * tb)) + 0.3f * __sinf((float)(6.283185307179586 * 120.0 * tb)) +
              0.1f * __sinf((float)(6.283185307179586 * 180.0 * tb))) *
             e;
    }
    const double th = t - (bi + 0.5) * beat;
    if (th >= 0.0 && th < 0.03) {
        const uint64_t r = splitmix(seed * 0x100000001B3ull ^ i);
        const float nz = (float)(r >> 40) * (1.0f / 8388608.0f) - 1.0f;
        x += nz * __expf(-(float)th * 60.0f) * 0.15f;
    }
    const int MAJ[7] = {0, 2, 4, 5, 7, 9, 11}, MIN[7] = {0, 2, 3, 5, 7, 8, 10};
    const int* sc = mode == 0 ? MAJ : MIN;
    const int root = 48 + tonic;
    const int triad[3] = {root, root + sc[2], root + sc[4]};
    for (int k = 0; k < 3; k++) {
        const float f = 440.0f * __powf(2.0f, (float)(triad[k] - 69) / 12.0f);
        x += (0.2f / 3.0f) * tone3(f, t);
    }
    const double step = beat / 2.0;
    const int64_t k8 = (int64_t)(t / step);
    const double tl = t - (double)k8 * step;
    const int deg = (int)(splitmix(seed ^ (0xABCDull + (uint64_t)k8)) % 7);
    const float fl = 440.0f * __powf(2.0f, (float)(root + 12 + sc[deg] - 69) / 12.0f);
    x += 0.2f * tone3(fl, t) * __expf(-(float)tl * 3.0f) / 1.5f;
    out[(uint64_t)trk * len + i] = x;
}

__global__ void k_scale(float* __restrict__ out, uint64_t len, const unsigned int* __restrict__ peak_bits) {
    const int trk = blockIdx.y;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const float pk = sd_from_bits_f(peak_bits[trk]);
    if (pk > 0.0f) out[(uint64_t)trk * len + i] *= 0.9f / pk;
}

__global__ void k_peak_plain(const float* __restrict__ x, uint64_t len, unsigned int* __restrict__ peak_bits) {
    const int trk = blockIdx.y;
    float m = 0.0f;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x)
        m = sd_maxf(m, sd_absf(x[(uint64_t)trk * len + i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0 && m > 0.0f) atomicMax(&peak_bits[trk], sd_bits_f(m));
}

void launch_synth(float* out, uint64_t n_tracks, uint64_t len, uint32_t sr, const float* bpm, const int* key,
                  uint64_t seed0, hipStream_t st) {
    if (n_tracks == 0 || len == 0) return;
    for (uint64_t t0 = 0; t0 < n_tracks; t0 += 32768) {
        const unsigned nt = (unsigned)((n_tracks - t0) < 32768 ? (n_tracks - t0) : 32768);
        dim3 grid((unsigned)((len + 255) / 256), nt);
        hipLaunchKernelGGL(k_synth, grid, dim3(256), 0, st, out + t0 * len, len, sr, bpm + t0, key + t0, seed0 + t0);
    }
}

void launch_synth_normalize(float* out, uint64_t n_tracks, uint64_t len, unsigned int* peak_bits, hipStream_t st) {
    if (n_tracks == 0 || len == 0) return;
    (void)hipMemsetAsync(peak_bits, 0, n_tracks * sizeof(unsigned int), st);
    for (uint64_t t0 = 0; t0 < n_tracks; t0 += 32768) {
        const unsigned nt = (unsigned)((n_tracks - t0) < 32768 ? (n_tracks - t0) : 32768);
        hipLaunchKernelGGL(k_peak_plain, dim3(64, nt), dim3(256), 0, st, out + t0 * len, len, peak_bits + t0);
        hipLaunchKernelGGL(k_scale, dim3((unsigned)((len + 255) / 256), nt), dim3(256), 0, st, out + t0 * len, len,
                           peak_bits + t0);
    }
}

}  // namespace sdsp
