// k_stft.hip — batched real-input STFT magnitudes for gfx950 (replaces compute_stft,
// reference src/features/chroma/extractor.rs:301-359, whose FFT is rustfft).
//
// Arithmetic: exactly sdsp_fft_spec.h (Stockham radix-4 DIF stages, real-FFT post-twiddle),
// so the spectra are bit-identical to the CPU restatement.  Data movement: two consecutive
// radix-4 stages touch a closed set of 16 elements (stage (n, s) butterflies
// p = p' + j'*n/16, j' = 0..3, feed stage (n/4, 4s) butterflies q + s*jA), so each thread
// runs both stages on 16 values held in registers ("radix-16 pass"): one LDS round trip per
// two stages instead of one per stage.
//
//   N = 8192 (M = 4096 = 16^3):       3 radix-16 passes, 256 threads per frame
//   N = 2048 (M = 1024 = 16^2 * 4):   2 radix-16 passes + 1 radix-4 pass, 64 threads (one
//                                     wave) per frame, 4 frames per workgroup
//
// The first pass reads the frame straight from HBM (x*gain*window, the reference's two f32
// multiplies); the post-twiddle pass writes |X[k]|, k = 0..M, as coalesced row segments.
// LDS index padding i + i/16 keeps the strided pass-1 stores near conflict-free.
//
// Ragged batches: the flat frame index (frame_pfx prefix sums) picks the track.  Frames are
// numbered XCD-contiguously (xcd_block) so the 16x (N=8192) / 4x (N=2048) overlap between
// neighbouring frames is served from one L2.
#include "kernels.hpp"

namespace sdsp {

__device__ __forceinline__ int lpad(int i) { return i + (i >> 4); }

__device__ __forceinline__ void bfly4(cx a, cx b, cx c, cx d, cx w1, cx w2, cx w3, cx& y0, cx& y1, cx& y2, cx& y3) {
    const cx apc = cadd(a, c), amc = csub(a, c);
    const cx bpd = cadd(b, d), bmd = csub(b, d);
    const cx jbmd = {bmd.im, -bmd.re};
    y0 = cadd(apc, bpd);
    y1 = cmul(w1, cadd(amc, jbmd));
    y2 = cmul(w2, csub(apc, bpd));
    y3 = cmul(w3, csub(amc, jbmd));
}

// Two radix-4 stages, (n, s) then (n/4, 4s), on v[j' + 4j] = x[q + s(p' + (n/16)(j' + 4j))].
// On return v[jA + 4jB] = z[q + 16 s p' + s(jA + 4jB)].
template <int M>
__device__ __forceinline__ void radix16(cx v[16], const cx* __restrict__ tw, int n, int pp) {
    const int m1 = n / 16;
    const int tA = M / n, tB = 4 * (M / n);
    cx u[16];
#pragma unroll
    for (int jp = 0; jp < 4; jp++) {
        const int p = pp + jp * m1;
        const cx w1 = tw[1 * p * tA], w2 = tw[2 * p * tA], w3 = tw[3 * p * tA];
        bfly4(v[jp], v[jp + 4], v[jp + 8], v[jp + 12], w1, w2, w3, u[jp * 4 + 0], u[jp * 4 + 1], u[jp * 4 + 2],
              u[jp * 4 + 3]);
    }
    const cx w1 = tw[1 * pp * tB], w2 = tw[2 * pp * tB], w3 = tw[3 * pp * tB];
#pragma unroll
    for (int ja = 0; ja < 4; ja++)
        bfly4(u[0 * 4 + ja], u[1 * 4 + ja], u[2 * 4 + ja], u[3 * 4 + ja], w1, w2, w3, v[ja + 0], v[ja + 4], v[ja + 8],
              v[ja + 12]);
}

template <int NFFT, bool FRAME_MAX>
__global__ __launch_bounds__(256) void k_stft_mag(const float* __restrict__ samples,
                                                  const uint64_t* __restrict__ frame_pfx, int n_tracks,
                                                  uint64_t total_frames, const uint64_t* __restrict__ src_off,
                                                  const float* __restrict__ gain, int hop,
                                                  const float* __restrict__ window, const cx* __restrict__ tw,
                                                  const cx* __restrict__ rt, float* __restrict__ mags,
                                                  const uint64_t* __restrict__ mag_row0, int stride,
                                                  float* __restrict__ frame_max) {
    constexpr int M = NFFT / 2;
    constexpr int TPF = M / 16;          // threads per frame (one radix-16 group each)
    constexpr int FPB = 256 / TPF;       // frames per workgroup
    constexpr int PADM = M + M / 16;     // padded LDS slots per frame
    static_assert(TPF == 64 || TPF == 256, "supported sizes: N = 2048, 8192");
    __shared__ cx lds[FPB * PADM];
    __shared__ float red[4];

    const int lt = threadIdx.x % TPF;            // thread within frame
    const int fl = threadIdx.x / TPF;            // frame within workgroup
    const uint64_t g = (uint64_t)xcd_block(blockIdx.x, gridDim.x) * FPB + fl;
    const bool live = g < total_frames;
    const uint64_t gg = live ? g : total_frames - 1;  // dead lanes recompute the last frame
    const int trk = find_track(frame_pfx, n_tracks, gg);
    const uint64_t f = gg - frame_pfx[trk];
    const float* x = samples + src_off[trk] + f * (uint64_t)hop;
    const float gn = gain[trk];
    cx* buf = lds + fl * PADM;

    cx v[16];
    // pass 1 (n = M, s = 1, p' = lt): z[idx] = (x[2idx], x[2idx+1]) * gain * window
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int idx = lt + TPF * k;
        const float s0 = x[2 * idx] * gn;
        const float s1 = x[2 * idx + 1] * gn;
        v[k] = {s0 * window[2 * idx], s1 * window[2 * idx + 1]};
    }
    radix16<M>(v, tw, M, lt);
#pragma unroll
    for (int k = 0; k < 16; k++) buf[lpad(16 * lt + k)] = v[k];
    __syncthreads();
    // further radix-16 passes
#pragma unroll
    for (int n = M / 16, s = 16; n >= 16; n /= 16, s *= 16) {
        const int q = lt % s, pp = lt / s;
        const int m1 = n / 16;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = buf[lpad(q + s * pp + s * m1 * k)];
        __syncthreads();
        radix16<M>(v, tw, n, pp);
#pragma unroll
        for (int k = 0; k < 16; k++) buf[lpad(q + 16 * s * pp + s * k)] = v[k];
        __syncthreads();
    }
    // trailing radix-4 stage (M = 16^k * 4): n = 4, s = M/4, p = 0
    if constexpr (M == 1024) {
        constexpr int s = M / 4;
        const cx w0 = tw[0];
#pragma unroll
        for (int r = 0; r < s / TPF; r++) {
            const int q = lt + TPF * r;
            cx y0, y1, y2, y3;
            bfly4(buf[lpad(q)], buf[lpad(q + s)], buf[lpad(q + 2 * s)], buf[lpad(q + 3 * s)], w0, w0, w0, y0, y1, y2,
                  y3);
            buf[lpad(q)] = y0;
            buf[lpad(q + s)] = y1;
            buf[lpad(q + 2 * s)] = y2;
            buf[lpad(q + 3 * s)] = y3;
        }
        __syncthreads();
    }
    // real-FFT post-processing, |X[k]|, k = 0..M
    float* out = mags + (mag_row0[trk] + f) * (uint64_t)stride;
    float mx = 0.0f;
    auto post = [&](int k, cx w) {
        const cx Zk = buf[lpad(k & (M - 1))];
        const cx Zr = buf[lpad((M - k) & (M - 1))];
        const cx Zc = {Zr.re, -Zr.im};
        const cx E = {(Zk.re + Zc.re) * 0.5f, (Zk.im + Zc.im) * 0.5f};
        const cx D = csub(Zk, Zc);
        const cx O = {D.im * 0.5f, -(D.re * 0.5f)};
        const cx X = cadd(E, cmul(w, O));
        const float mag = __builtin_sqrtf(X.re * X.re + X.im * X.im);
        if (live) out[k] = mag;
        if (FRAME_MAX) mx = sd_maxf(mx, mag);
    };
    // k = lt + TPF*j for j < M/TPF (post twiddles loaded up front), then k = M on lane 0
    constexpr int NPOST = M / TPF;
    cx wr[NPOST];
#pragma unroll
    for (int j = 0; j < NPOST; j++) wr[j] = rt[lt + TPF * j];
#pragma unroll
    for (int j = 0; j < NPOST; j++) post(lt + TPF * j, wr[j]);
    if (lt == 0) post(M, rt[M]);
    if (FRAME_MAX) {
        if constexpr (TPF == 64) {
            mx = wave_max(mx);
            if (lt == 0 && live) frame_max[mag_row0[trk] + f] = mx;
        } else {
            mx = wave_max(mx);
            if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
            __syncthreads();
            if (threadIdx.x == 0 && live) {
                float m = red[0];
                for (int i = 1; i < 4; i++) m = sd_maxf(m, red[i]);
                frame_max[mag_row0[trk] + f] = m;
            }
        }
    }
}

// host launcher (the runtime owns all buffers; see runtime.hip)
void launch_stft(int nfft, bool frame_max, const float* samples, const uint64_t* frame_pfx, int n_tracks,
                 uint64_t total_frames, const uint64_t* src_off, const float* gain, int hop, const float* window,
                 const cx* tw, const cx* rt, float* mags, const uint64_t* mag_row0, int stride, float* fmax,
                 hipStream_t st) {
    if (total_frames == 0) return;
    const dim3 block(256);
    if (nfft == 2048) {
        const dim3 grid((unsigned)((total_frames + 3) / 4));
        if (frame_max)
            hipLaunchKernelGGL((k_stft_mag<2048, true>), grid, block, 0, st, samples, frame_pfx, n_tracks,
                               total_frames, src_off, gain, hop, window, tw, rt, mags, mag_row0, stride, fmax);
        else
            hipLaunchKernelGGL((k_stft_mag<2048, false>), grid, block, 0, st, samples, frame_pfx, n_tracks,
                               total_frames, src_off, gain, hop, window, tw, rt, mags, mag_row0, stride, fmax);
    } else if (nfft == 8192) {
        hipLaunchKernelGGL((k_stft_mag<8192, false>), dim3((unsigned)total_frames), block, 0, st, samples, frame_pfx,
                           n_tracks, total_frames, src_off, gain, hop, window, tw, rt, mags, mag_row0, stride, fmax);
    }
}

}  // namespace sdsp
