// k_features.hip — every per-frame reduction of the 2048-point magnitude spectrogram in one
// pass over HBM (reference src/features/period/novelty.rs and src/features/onset/*):
//
//   E[v][t]   = sum_k |X_t[k]|^2 over band v          energy_flux_novelty(_band)  novelty.rs:504-508,641-644
//   H[v][t]   = sum_k (k*|X_t[k]|)*|X_t[k]|           hfc_novelty(_band) / detect_hfc_onsets  :738-747,810-821, hfc.rs:130-137
//   SFX[v][t] = sqrt(sum_k max(0, L_t[k] - max_{|j-k|<=K, j in band} L_{t-1}[j])^2)   superflux(_band) :353-376,419-442
//   SFO[t]    = sqrt(sum_k max(0, X_t[k]/max_t - X_{t-1}[k]/max_{t-1})^2)            spectral_flux.rs:116-157
//   MEL[t][m] = sum_k L_t[k] * w_{k,m}  (HTK triangles, bins ascending)               MelFilterbank::apply_logmag :174-190
//   with L = ln(1 + max(X, 0)), v in {full, low, mid, high}.
//
// Each workgroup owns 128 consecutive frames of one track, one thread per frame.  Bins are
// streamed in 32-bin chunks: the workgroup stages rows t-1..t+127 of the chunk into LDS with
// coalesced 128-B row segments (log values computed once per element, with a +-K halo for
// the SuperFlux max filter), then each thread walks its frame's bins *in order*, so every f32
// accumulation happens in exactly the reference's sequence and the results are bit-identical
// to the CPU restatement.  Band membership is uniform across the workgroup (all threads
// visit the same bin at the same time), so the band logic never diverges.
#include "kernels.hpp"

namespace sdsp {

constexpr int FT_CW = 32;

__global__ __launch_bounds__(FT_FRAMES) void k_features(const float* __restrict__ mags,
                                                        const float* __restrict__ fmax,
                                                        const uint64_t* __restrict__ frame_pfx,
                                                        const uint64_t* __restrict__ tile_pfx, int T, FeatParams P,
                                                        const int* __restrict__ mel_m, const float* __restrict__ mel_w,
                                                        float* __restrict__ E, float* __restrict__ H,
                                                        float* __restrict__ SFX, float* __restrict__ SFO,
                                                        float* __restrict__ MEL, uint64_t total) {
    __shared__ float Mt[FT_FRAMES + 1][FT_CW + 1];
    __shared__ float Lt[FT_FRAMES + 1][FT_CW + 2 * FT_KMAX + 1];
    __shared__ float melacc[FT_MELMAX][FT_FRAMES];

    const uint64_t gb = blockIdx.x;
    const int trk = find_track(tile_pfx, T, gb);
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[trk]) * FT_FRAMES;
    const uint64_t g0 = frame_pfx[trk];
    const int i = threadIdx.x;
    const int64_t f = f0 + i;
    const bool valid = f < F;
    const bool has_prev = valid && f >= 1;
    const int K = P.K, B = P.B;

    for (int m = 0; m < P.n_mels; m++) melacc[m][i] = 0.0f;
    float e[4] = {0, 0, 0, 0}, h[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0}, so = 0.0f;
    const float mx_c = valid ? fmax[g0 + f] : 0.0f;
    const float mx_p = has_prev ? fmax[g0 + f - 1] : 0.0f;
    const bool cn = mx_c > EPS, pn = mx_p > EPS;

    for (int c0 = 0; c0 < B; c0 += FT_CW) {
        __syncthreads();
        // stage rows f0-1 .. f0+127 of [c0-K, c0+CW+K)
        const int LW = FT_CW + 2 * K;
        for (int idx = i; idx < (FT_FRAMES + 1) * LW; idx += FT_FRAMES) {
            const int r = idx / LW, j = idx - r * LW;
            const int64_t fr = f0 - 1 + r;
            const int b = c0 - K + j;
            float v = 0.0f;
            if (fr >= 0 && fr < F && b >= 0 && b < B) v = mags[(g0 + (uint64_t)fr) * (uint64_t)P.stride + b];
            Lt[r][j] = sd_logf(1.0f + sd_maxf(v, 0.0f));
            if (j >= K && j < K + FT_CW) Mt[r][j - K] = v;
        }
        __syncthreads();
        if (!valid) continue;
        const int nb = B - c0 < FT_CW ? B - c0 : FT_CW;
        for (int j = 0; j < nb; j++) {
            const int b = c0 + j;
            const float m = Mt[i + 1][j];
            const float ee = m * m;
            const float hh = (float)b * m * m;
            e[0] += ee;
            h[0] += hh;
#pragma unroll
            for (int v = 1; v < 4; v++)
                if (P.band_on[v] && b >= P.bs[v] && b < P.be[v]) {
                    e[v] += ee;
                    h[v] += hh;
                }
            const float lc = Lt[i + 1][j + K];
            // mel accumulation, contributions in ascending mel index (novelty.rs:181-186)
            if (lc > 0.0f) {
                const int m1 = mel_m[2 * b], m2 = mel_m[2 * b + 1];
                if (m1 >= 0) melacc[m1][i] += lc * mel_w[2 * b];
                if (m2 >= 0) melacc[m2][i] += lc * mel_w[2 * b + 1];
            }
            if (has_prev) {
                const float mp = Mt[i][j];
                const float pv = pn ? mp / mx_p : 0.0f;
                const float cv = cn ? m / mx_c : 0.0f;
                const float d = sd_maxf(cv - pv, 0.0f);
                so += d * d;
                // SuperFlux, full band window [b-K, b+K] clipped to [0, B)
                const int lo = b - K < 0 ? 0 : b - K;
                const int hi = b + K + 1 < B ? b + K + 1 : B;
                float pm = 0.0f;
                for (int q = lo; q < hi; q++) pm = sd_maxf(pm, Lt[i][q - c0 + K]);
                const float df = sd_maxf(lc - pm, 0.0f);
                sx[0] += df * df;
#pragma unroll
                for (int v = 1; v < 4; v++) {
                    if (P.band_on[v] && b >= P.bs[v] && b < P.be[v]) {
                        float pmb = pm;
                        if (lo < P.bs[v] || hi > P.be[v]) {
                            const int lb = lo < P.bs[v] ? P.bs[v] : lo;
                            const int hb = hi > P.be[v] ? P.be[v] : hi;
                            pmb = 0.0f;
                            for (int q = lb; q < hb; q++) pmb = sd_maxf(pmb, Lt[i][q - c0 + K]);
                        }
                        const float db = sd_maxf(lc - pmb, 0.0f);
                        sx[v] += db * db;
                    }
                }
            }
        }
    }
    if (!valid) return;
    const uint64_t g = g0 + (uint64_t)f;
#pragma unroll
    for (int v = 0; v < 4; v++) {
        E[(uint64_t)v * total + g] = e[v];
        H[(uint64_t)v * total + g] = h[v];
    }
    for (int m = 0; m < P.n_mels; m++) MEL[g * (uint64_t)P.n_mels + m] = melacc[m][i];
    if (has_prev) {
        const uint64_t gp = g - 1;  // pair (t-1, t) stored at t-1
        SFO[gp] = __builtin_sqrtf(so);
#pragma unroll
        for (int v = 0; v < 4; v++) SFX[(uint64_t)v * total + gp] = __builtin_sqrtf(sx[v]);
    }
}

void launch_features(const float* mags, const float* fmax, const uint64_t* frame_pfx, const uint64_t* tile_pfx,
                     int T, uint64_t n_tiles, const FeatParams& P, const int* mel_m, const float* mel_w, float* E,
                     float* H, float* SFX, float* SFO, float* MEL, uint64_t total, hipStream_t st) {
    if (n_tiles == 0) return;
    hipLaunchKernelGGL(k_features, dim3((unsigned)n_tiles), dim3(FT_FRAMES), 0, st, mags, fmax, frame_pfx, tile_pfx,
                       T, P, mel_m, mel_w, E, H, SFX, SFO, MEL, total);
}

}  // namespace sdsp
