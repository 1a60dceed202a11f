// k_novelty.hip — novelty curves from the per-frame features (reference
// src/features/period/novelty.rs:336-986):
//
//   variants full/low/mid/high:  combined_novelty_with_params(superflux, energy flux, HFC flux)
//       normalise each flux (:383-386, :521-530, :757-766), weighted mix / wsum (:893-904),
//       normalise, local-mean subtraction with half-wave rectification (:943-964),
//       moving average (:966-983), normalise.
//   variant mel:  mel SuperFlux (:574-608), normalised.
//
// One workgroup per (track, variant); curves live in L2-resident global scratch between the
// phases (every phase is elementwise or a short in-order window sum, so all outputs keep the
// reference's exact f32 operation order; maxima are order-free).  The last phase also
// produces the curve's sequential sum, used as the FFT tempogram's DC removal
// (tempogram_fft.rs:110).
#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdsp {

__global__ __launch_bounds__(1024) void k_novelty(const float* __restrict__ E, const float* __restrict__ H,
                                                   const float* __restrict__ SFX, const uint64_t* __restrict__ frame_pfx,
                                                   int T, uint64_t total, NovParams P, float* __restrict__ scratch,
                                                   float* __restrict__ nov, float* __restrict__ nov_sum) {
    SDSP_LATENCY_CRITICAL();
    __shared__ float red[16];
    const int trk = blockIdx.x % T, v = blockIdx.x / T;
    if (!P.band_on[v]) return;
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    if (F < 2) return;
    const int64_t L = F - 1;
    const uint64_t g0 = frame_pfx[trk];
    const float* e = E + (uint64_t)v * total + g0;
    const float* h = H + (uint64_t)v * total + g0;
    const float* s = SFX + (uint64_t)v * total + g0;
    float* A = scratch + ((uint64_t)v * 2 + 0) * total + g0;
    float* Bf = scratch + ((uint64_t)v * 2 + 1) * total + g0;
    float* out = nov + (uint64_t)v * total + g0;
    const int tid = threadIdx.x, NT = blockDim.x;

    float ms = 0.0f, me = 0.0f, mh = 0.0f;
    for (int64_t i = tid; i < L; i += NT) {
        ms = sd_maxf(ms, s[i]);
        me = sd_maxf(me, sd_maxf(e[i + 1] - e[i], 0.0f));
        mh = sd_maxf(mh, sd_maxf(h[i + 1] - h[i], 0.0f));
    }
    ms = block_max(ms, red);
    me = block_max(me, red);
    mh = block_max(mh, red);
    float mc = 0.0f;
    for (int64_t i = tid; i < L; i += NT) {
        float sv = s[i], ev = sd_maxf(e[i + 1] - e[i], 0.0f), hv = sd_maxf(h[i + 1] - h[i], 0.0f);
        if (ms > EPS) sv /= ms;
        if (me > EPS) ev /= me;
        if (mh > EPS) hv /= mh;
        const float c = (sv * P.ws + ev * P.we + hv * P.wh) / P.wsum;
        A[i] = c;
        mc = sd_maxf(mc, c);
    }
    mc = block_max(mc, red);
    if (mc > EPS)
        for (int64_t i = tid; i < L; i += NT) A[i] /= mc;
    __syncthreads();
    float* cur = A;
    float* oth = Bf;
    if (P.lmw > 1) {
        const int64_t half = P.lmw / 2;
        for (int64_t i = tid; i < L; i += NT) {
            const int64_t st = i >= half ? i - half : 0;
            const int64_t en = i + half + 1 < L ? i + half + 1 : L;
            float sum = 0.0f;
            for (int64_t j = st; j < en; j++) sum += cur[j];
            const float mean = sum / (float)(en - st);
            oth[i] = sd_maxf(cur[i] - mean, 0.0f);
        }
        __syncthreads();
        float* t = cur;
        cur = oth;
        oth = t;
    }
    if (P.smw > 1 && L >= 3) {
        const int64_t half = P.smw / 2;
        for (int64_t i = tid; i < L; i += NT) {
            const int64_t st = i >= half ? i - half : 0;
            const int64_t en = i + half + 1 < L ? i + half + 1 : L;
            float sum = 0.0f;
            for (int64_t j = st; j < en; j++) sum += cur[j];
            oth[i] = sum / (float)(en - st);
        }
        __syncthreads();
        float* t = cur;
        cur = oth;
        oth = t;
    }
    float mf = 0.0f;
    for (int64_t i = tid; i < L; i += NT) mf = sd_maxf(mf, cur[i]);
    mf = block_max(mf, red);
    for (int64_t i = tid; i < L; i += NT) out[i] = mf > EPS ? cur[i] / mf : cur[i];
    __syncthreads();
    __shared__ float sbuf[SEQ_CH];
    const float sum = block_seq_sum(out, L, sbuf);
    if (tid == 0) nov_sum[(uint64_t)v * T + trk] = sum;
}

// mel SuperFlux novelty (novelty.rs:553-609), variant index 4, in two kernels:
// k_mel_flux, one thread per frame pair over the whole batch (MEL is mel-major, so the
// reads are coalesced), raw flux + per-track max (atomicMax on the bits of a value >= 0);
// k_mel_norm, one workgroup per track: normalise, then the curve's sequential sum.
__device__ inline float mel_flux_frame(const float* mtile, int RW, int i, int n_mels, int K) {
    float sum = 0.0f;
    if (K == 2) {
        // the default: the previous frame's mels in a 5-register window (one LDS read per mel
        // instead of five).  Mel sums are >= +0 and never NaN, so the window's +0 padding past
        // either end leaves every maximum (from +0, over the clipped range) unchanged.
        float w0 = 0.0f, w1 = 0.0f, w2 = mtile[i], w3 = n_mels > 1 ? mtile[RW + i] : 0.0f;
        for (int b = 0; b < n_mels; b++) {
            const float w4 = b + 2 < n_mels ? mtile[(b + 2) * RW + i] : 0.0f;
            const float pm = sd_maxf(sd_maxf(sd_maxf(sd_maxf(sd_maxf(0.0f, w0), w1), w2), w3), w4);
            const float d = sd_maxf(mtile[b * RW + i + 1] - pm, 0.0f);
            sum += d * d;
            w0 = w1;
            w1 = w2;
            w2 = w3;
            w3 = w4;
        }
        return __builtin_sqrtf(sum);
    }
    for (int b = 0; b < n_mels; b++) {
        const int lo = b - K < 0 ? 0 : b - K;
        const int hi = b + K + 1 < n_mels ? b + K + 1 : n_mels;
        float pm = 0.0f;
        for (int q = lo; q < hi; q++) pm = sd_maxf(pm, mtile[q * RW + i]);
        const float d = sd_maxf(mtile[b * RW + i + 1] - pm, 0.0f);
        sum += d * d;
    }
    return __builtin_sqrtf(sum);
}

__global__ __launch_bounds__(256) void k_mel_flux(const float* __restrict__ MEL, int n_mels, int K,
                                                  const uint64_t* __restrict__ frame_pfx, int T, uint64_t total,
                                                  float* __restrict__ nov, unsigned int* __restrict__ mx_bits) {
    SDSP_LATENCY_CRITICAL();
    extern __shared__ float mtile[];  // [n_mels][257]: frames gb .. gb+256
    constexpr int RW = 257;
    const uint64_t gb = (uint64_t)blockIdx.x * 256;
    // 8 mel rows in flight per thread (the loads of a batch before its LDS stores)
    for (int m0 = 0; m0 < n_mels; m0 += 8)
        for (int r = threadIdx.x; r < RW; r += 256) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; k++)
                v[k] = (m0 + k < n_mels && gb + r < total) ? MEL[(uint64_t)(m0 + k) * total + gb + r] : 0.0f;
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (m0 + k < n_mels) mtile[(m0 + k) * RW + r] = v[k];
        }
    __syncthreads();
    const int i = threadIdx.x;
    const uint64_t g = gb + i;
    const int trk = g < total ? find_track(frame_pfx, T, g) : -1;
    // frames without a successor in their track (and padding lanes) contribute 0 to the max
    float fl = 0.0f;
    if (trk >= 0 && g + 1 < frame_pfx[trk + 1]) {
        fl = mel_flux_frame(mtile, RW, i, n_mels, K);
        nov[4 * total + g] = fl;
    }
    // one atomic per wave when the wave lies in one track (the common case)
    const int t0 = __shfl(trk, 0, 64);
    if (__all(trk == t0)) {
        const float wm = wave_max(fl);
        if ((threadIdx.x & 63) == 0 && t0 >= 0 && wm > 0.0f) atomicMax(&mx_bits[t0], sd_bits_f(wm));
    } else if (trk >= 0 && fl > 0.0f) {
        atomicMax(&mx_bits[trk], sd_bits_f(fl));
    }
}


__global__ __launch_bounds__(256) void k_mel_norm(const uint64_t* __restrict__ frame_pfx, int T, uint64_t total,
                                                  const unsigned int* __restrict__ mx_bits, float* __restrict__ nov,
                                                  float* __restrict__ nov_sum) {
    SDSP_LATENCY_CRITICAL();
    __shared__ float sbuf[SEQ_CH];
    const int trk = blockIdx.x;
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    if (F < 2) return;
    const int64_t L = F - 1;
    float* out = nov + 4 * total + frame_pfx[trk];
    const float mf = sd_from_bits_f(mx_bits[trk]);
    if (mf > EPS)
        for (int64_t i = threadIdx.x; i < L; i += blockDim.x) out[i] /= mf;
    __syncthreads();
    const float sum = block_seq_sum(out, L, sbuf);
    if (threadIdx.x == 0) nov_sum[4 * (uint64_t)T + trk] = sum;
}

void launch_novelty(const float* E, const float* H, const float* SFX, const uint64_t* frame_pfx, int T, uint64_t total,
                    const NovParams& P, float* scratch, float* nov, float* nov_sum, const float* MEL, int n_mels,
                    int mel_k, bool mel_on, unsigned int* mel_max, hipStream_t st) {
    if (T == 0) return;
    hipLaunchKernelGGL(k_novelty, dim3(4 * T), dim3(1024), 0, st, E, H, SFX, frame_pfx, T, total, P, scratch, nov,
                       nov_sum);
    if (mel_on && total > 0) {
        (void)hipMemsetAsync(mel_max, 0, (size_t)T * sizeof(unsigned int), st);
        hipLaunchKernelGGL(k_mel_flux, dim3((unsigned)((total + 255) / 256)), dim3(256),
                           (size_t)n_mels * 257 * sizeof(float), st, MEL, n_mels, mel_k,
                           frame_pfx, T, total, nov, mel_max);
        hipLaunchKernelGGL(k_mel_norm, dim3(T), dim3(256), 0, st, frame_pfx, T, total, mel_max, nov, nov_sum);
    }
}

}  // namespace sdsp
