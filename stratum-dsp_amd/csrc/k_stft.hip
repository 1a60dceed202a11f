// k_stft.hip — batched real-input STFT magnitudes for gfx950 (replaces compute_stft,
// reference src/features/chroma/extractor.rs:301-359, whose FFT is rustfft).
//
// One 256-thread workgroup (4 waves) per frame.  The frame's N real samples are read once
// from HBM straight into registers (stage 0 of the Stockham pass reads global memory; the
// reference's peak-normalisation gain and symmetric Hann window are applied on the fly as
// two f32 multiplies, (x*gain)*w, exactly as the reference materialises them), the N/2-point
// complex FFT runs radix-4 Stockham through one LDS buffer, and the real-FFT post-twiddle
// writes |X[k]| for k = 0..N/2 with 16-B-aligned rows.  Arithmetic order == sdsp_fft_spec.h,
// so the result is bit-identical to the CPU restatement.
//
// Ragged batches: blockIdx.x is a flat frame index over all tracks (frame_pfx prefix sums).
#include "kernels.hpp"

namespace sdsp {

template <int NFFT, bool FRAME_MAX>
__global__ __launch_bounds__(256) void k_stft_mag(const float* __restrict__ samples,
                                                  const uint64_t* __restrict__ frame_pfx, int n_tracks,
                                                  const uint64_t* __restrict__ src_off,
                                                  const float* __restrict__ gain, int hop,
                                                  const float* __restrict__ window, const cx* __restrict__ tw,
                                                  const cx* __restrict__ rt, float* __restrict__ mags,
                                                  const uint64_t* __restrict__ mag_row0, int stride,
                                                  float* __restrict__ frame_max) {
    constexpr int NT = 256;
    constexpr int M = NFFT / 2;
    constexpr int NBF = M / 4 / NT;  // radix-4 butterflies per thread per stage
    static_assert(NBF >= 1, "NFFT too small for 256 threads");
    constexpr int LOG4 = (M == 1024) ? 5 : (M == 4096) ? 6 : (M == 256) ? 4 : 0;
    static_assert(LOG4 > 0, "M must be a power of 4 in {256, 1024, 4096}");
    __shared__ cx buf[M];
    __shared__ float red[NT / WAVE];

    const uint64_t g = blockIdx.x;
    const int trk = find_track(frame_pfx, n_tracks, g);
    const uint64_t f = g - frame_pfx[trk];
    const float* x = samples + src_off[trk] + f * (uint64_t)hop;
    const float gn = gain[trk];
    const int t = threadIdx.x;

    cx a[NBF][4];
    // stage-0 inputs: z[idx] = (x[2idx], x[2idx+1]) * gain * window
#pragma unroll
    for (int r = 0; r < NBF; r++) {
        const int p = t + NT * r;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int idx = p + j * (M / 4);
            const float s0 = x[2 * idx] * gn;
            const float s1 = x[2 * idx + 1] * gn;
            a[r][j] = {s0 * window[2 * idx], s1 * window[2 * idx + 1]};
        }
    }
    int n = M, s = 1;
#pragma unroll
    for (int st = 0; st < LOG4; st++) {
        const int m = n / 4;
        const int tstep = M / n;
        cx y[NBF][4];
        int pp[NBF], qq[NBF];
#pragma unroll
        for (int r = 0; r < NBF; r++) {
            const int beta = t + NT * r;
            const int p = beta / s, q = beta - p * s;
            pp[r] = p;
            qq[r] = q;
            const cx w1 = tw[1 * p * tstep], w2 = tw[2 * p * tstep], w3 = tw[3 * p * tstep];
            const cx apc = cadd(a[r][0], a[r][2]), amc = csub(a[r][0], a[r][2]);
            const cx bpd = cadd(a[r][1], a[r][3]), bmd = csub(a[r][1], a[r][3]);
            const cx jbmd = {bmd.im, -bmd.re};
            y[r][0] = cadd(apc, bpd);
            y[r][1] = cmul(w1, cadd(amc, jbmd));
            y[r][2] = cmul(w2, csub(apc, bpd));
            y[r][3] = cmul(w3, csub(amc, jbmd));
        }
        if (st > 0) __syncthreads();  // every thread has read this stage's inputs
#pragma unroll
        for (int r = 0; r < NBF; r++)
#pragma unroll
            for (int j = 0; j < 4; j++) buf[qq[r] + s * (4 * pp[r] + j)] = y[r][j];
        __syncthreads();
        n = m;
        s *= 4;
        if (st + 1 < LOG4) {
            const int m2 = n / 4;
#pragma unroll
            for (int r = 0; r < NBF; r++) {
                const int beta = t + NT * r;
                const int p = beta / s, q = beta - p * s;
#pragma unroll
                for (int j = 0; j < 4; j++) a[r][j] = buf[q + s * (p + j * m2)];
            }
        }
    }
    // real-FFT post-processing, |X[k]|, k = 0..M
    float* out = mags + (mag_row0[trk] + f) * (uint64_t)stride;
    float mx = 0.0f;
    for (int k = t; k <= M; k += NT) {
        const cx Zk = buf[k & (M - 1)];
        const cx Zr = buf[(M - k) & (M - 1)];
        const cx Zc = {Zr.re, -Zr.im};
        const cx E = {(Zk.re + Zc.re) * 0.5f, (Zk.im + Zc.im) * 0.5f};
        const cx D = csub(Zk, Zc);
        const cx O = {D.im * 0.5f, -(D.re * 0.5f)};
        const cx X = cadd(E, cmul(rt[k], O));
        const float mag = __builtin_sqrtf(X.re * X.re + X.im * X.im);
        out[k] = mag;
        if (FRAME_MAX) mx = sd_maxf(mx, mag);
    }
    if (FRAME_MAX) {
        mx = wave_max(mx);
        if ((t & 63) == 0) red[t >> 6] = mx;
        __syncthreads();
        if (t == 0) {
            float v = red[0];
            for (int i = 1; i < NT / WAVE; i++) v = sd_maxf(v, red[i]);
            frame_max[mag_row0[trk] + f] = v;
        }
    }
}

// host launcher (the runtime owns all buffers; see runtime.hip)
void launch_stft(int nfft, bool frame_max, const float* samples, const uint64_t* frame_pfx, int n_tracks,
                 uint64_t total_frames, const uint64_t* src_off, const float* gain, int hop, const float* window,
                 const cx* tw, const cx* rt, float* mags, const uint64_t* mag_row0, int stride, float* fmax,
                 hipStream_t st) {
    if (total_frames == 0) return;
    dim3 grid((unsigned)total_frames), block(256);
    if (nfft == 2048 && frame_max)
        hipLaunchKernelGGL((k_stft_mag<2048, true>), grid, block, 0, st, samples, frame_pfx, n_tracks, src_off, gain,
                           hop, window, tw, rt, mags, mag_row0, stride, fmax);
    else if (nfft == 2048)
        hipLaunchKernelGGL((k_stft_mag<2048, false>), grid, block, 0, st, samples, frame_pfx, n_tracks, src_off, gain,
                           hop, window, tw, rt, mags, mag_row0, stride, fmax);
    else if (nfft == 8192)
        hipLaunchKernelGGL((k_stft_mag<8192, false>), grid, block, 0, st, samples, frame_pfx, n_tracks, src_off, gain,
                           hop, window, tw, rt, mags, mag_row0, stride, fmax);
}

}  // namespace sdsp
