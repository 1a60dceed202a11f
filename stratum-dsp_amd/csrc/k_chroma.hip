// k_chroma.hip — the key path's opt-in chroma front-ends (reference src/lib.rs:1062-1198):
//
//   k_tuning     global tuning offset per track           chroma/extractor.rs:66-177
//   k_chroma     frame_to_chroma_tuned per frame           extractor.rs:393-481, 1047-1094
//                log-frequency chroma per frame            extractor.rs:701-828, 937-985, lib.rs:1120-1131
//   k_hpcp_x     HPCP with tuning, whitening, bass blend   extractor.rs:529-680, 1097-1244
//   k_beat_sync  beat-synchronous chroma rows              extractor.rs:830-935
//
// Every per-frame kernel is one thread per frame, HP_FRAMES frames per workgroup, with the
// bins staged through LDS in coalesced HP_CW-column chunks (the k_hpcp layout); each thread
// folds its frame's bins in the reference's order.  Per-bin constants that depend on the
// track's tuning (pitch-class targets and Gaussian weights) are built once per workgroup in
// LDS.  Pitch-class accumulators live in LDS ([class][thread]: conflict-free).
#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdsp {

namespace {

constexpr int CW = 16;  // bins per staged chunk (LDS row stride CW + 1)
constexpr float TWO_PI_F = 2.0f * 3.14159265358979323846f;

// frame_to_chroma_tuned's per-bin pitch-class mapping (extractor.rs:420-470)
__device__ inline void chroma_bin_map(float f, float tuning, int soft, float sigma_in, int* tc0, float* w3) {
    const float semitone = 12.0f * sd_log2f(f / 440.0f) + 57.0f - tuning;
    if (soft) {
        const float spc = sd_rem_euclid_f(semitone, 12.0f);
        const float ppc = sd_rem_euclid_f(sd_roundf(spc), 12.0f);
        const int32_t primary = sd_f2i32(ppc);
        *tc0 = primary;
        for (int o = -1; o <= 1; o++) {
            const int tc = (((primary + o) % 12) + 12) % 12;
            float dist = sd_absf(spc - (float)tc);
            dist = sd_minf(dist, 12.0f - dist);
            const float sigma = sd_maxf(sigma_in, 1e-6f);
            w3[o + 1] = sd_expf(-dist * dist / (2.0f * sigma * sigma));
        }
    } else {
        int32_t cls = sd_f2i32(sd_roundf(semitone)) % 12;
        if (cls < 0) cls += 12;
        *tc0 = cls;
        w3[0] = w3[1] = w3[2] = 0.0f;
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// k_tuning: one workgroup per track.  Sampled frames (every `step`) are processed CHF at a time:
// the block takes each frame's in-band peak (order-free max), then every thread evaluates the
// (w sin, w cos, w) terms of its bins into LDS; lanes 0..2 of wave 0 fold the terms in
// (frame, bin) order — the reference's sequential f32 sums.
constexpr int TU_T = 256;
constexpr int TU_CHF = 8;
constexpr int TU_BAND_MAX = 1024;
__global__ __launch_bounds__(TU_T) void k_tuning(const float* __restrict__ mags, const uint64_t* __restrict__ frame_pfx,
                                                 const int* __restrict__ tracks, TuningParams P, float* __restrict__ out) {
    __shared__ float terms[3][TU_CHF * TU_BAND_MAX / 2];
    __shared__ float red[TU_T / 64];
    const int it = blockIdx.x;
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const float* base = mags + frame_pfx[trk] * (uint64_t)P.stride;
    const int TB = P.hi - P.lo + 1;
    const int chf = P.chf;  // frames per LDS batch (chf * TB <= capacity)
    float acc = 0.0f;       // lane 0: sum_sin, lane 1: sum_cos, lane 2: sum_w
    for (int64_t t0 = 0; t0 < F; t0 += (int64_t)chf * P.step) {
        int nt = 0;
        for (int q = 0; q < chf; q++) {
            const int64_t t = t0 + (int64_t)q * P.step;
            if (t >= F) break;
            const float* row = base + (uint64_t)t * (uint64_t)P.stride;
            float pk = 0.0f;
            for (int j = threadIdx.x; j < TB; j += TU_T) pk = sd_maxf(pk, row[P.lo + j]);
            const float peak = block_max(pk, red);
            const bool ok = !(peak <= 1e-12f);
            const float abs_thr = peak * P.thr;
            for (int j = threadIdx.x; j < TB; j += TU_T) {
                const int b = P.lo + j;
                const float m = row[b];
                float ws = 0.0f, wc = 0.0f, ww = 0.0f;
                if (ok && !(m < abs_thr)) {
                    const float f = (float)b * P.fres;
                    const float semitone = 12.0f * sd_log2f(f / 440.0f) + 57.0f;
                    const float residual = semitone - sd_roundf(semitone);
                    const float w = sd_powf(sd_maxf(m, 0.0f), 0.5f);
                    if (w > 0.0f) {
                        const float angle = TWO_PI_F * residual;
                        ws = w * sd_sinf(angle);
                        wc = w * sd_cosf(angle);
                        ww = w;
                    }
                }
                terms[0][nt * TB + j] = ws;
                terms[1][nt * TB + j] = wc;
                terms[2][nt * TB + j] = ww;
            }
            nt++;
        }
        __syncthreads();
        if (threadIdx.x < 3) {
            const float* tp = terms[threadIdx.x];
            const int n = nt * TB;
            for (int k = 0; k < n; k++) acc += tp[k];  // a skipped term is +-0: the sum is unchanged
        }
        __syncthreads();
    }
    __shared__ float sums[3];
    if (threadIdx.x < 3) sums[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float ss = sums[0], sc = sums[1], sw = sums[2];
        float d = 0.0f;
        if (!(sw <= 1e-6f)) {
            const float r = __builtin_sqrtf(ss * ss + sc * sc) / sw;
            if (!(r < 0.05f)) d = sd_atan2f(ss, sc) / TWO_PI_F;
        }
        out[it] = sd_clampf(d, -P.lim, P.lim);
    }
}

// ---------------------------------------------------------------------------------------------
// k_chroma: MODE 0 frame_to_chroma_tuned (+ raw energies), MODE 1 log-frequency chroma (+ the
// log-frequency energies).  The log-frequency spectrum is never stored: linear bins arrive in
// frequency order, so their semitone bins are non-decreasing and each semitone bin is final
// once a later linear bin maps past it; it is then folded into the chroma and the energy in
// semitone order (two accumulators: semitone bins L and L + 1).
template <int MODE>
__global__ __launch_bounds__(HP_FRAMES) void k_chroma(const float* __restrict__ mags,
                                                      const uint64_t* __restrict__ frame_pfx,
                                                      const uint64_t* __restrict__ tile_pfx,
                                                      const int* __restrict__ tracks, int n_items, ChromaParams P,
                                                      const float* __restrict__ tuning, float* __restrict__ chroma,
                                                      float* __restrict__ energy) {
    __shared__ float tile[HP_FRAMES][CW + 1];
    __shared__ float pc[12][HP_FRAMES];
    extern __shared__ ChromaBin tab[];  // [hi - lo + 1]
    const uint64_t gb = blockIdx.x;
    const int it = find_track(tile_pfx, n_items, gb);
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[it]) * HP_FRAMES;
    const int i = threadIdx.x;
    const int64_t f = f0 + i;
    const bool valid = f < F;
    const uint64_t g0 = frame_pfx[trk];
    // per-bin table for this track
    float tu = tuning ? tuning[it] : 0.0f;
    if (P.gate_small && !(sd_absf(tu) > 1e-6f)) tu = 0.0f;  // src/lib.rs:1178 (|offset| > 1e-6 or untuned)
    const int nb = P.hi - P.lo + 1;
    for (int j = i; j < nb; j += HP_FRAMES) {
        const int b = P.lo + j;
        const float fq = (float)b * P.fres;
        ChromaBin e{};
        if (MODE == 0) {
            float w3[3];
            chroma_bin_map(fq, tu, P.soft, P.sigma, &e.a, w3);
            e.w0 = w3[0], e.w1 = w3[1], e.w2 = w3[2];
        } else {
            const float semitone = 12.0f * sd_log2f(fq / 440.0f) + 57.0f;
            const float sf = semitone - (float)P.bmin;
            const uint64_t lo = sd_f2u64(__builtin_floorf(sf));
            uint64_t hi = sd_f2u64(__builtin_ceilf(sf));
            if (hi > (uint64_t)(P.n_log - 1)) hi = (uint64_t)(P.n_log - 1);
            const float wh = sf - (float)lo;
            e.a = lo < (uint64_t)P.n_log ? (int)lo : -1;
            e.b = (int)hi;
            e.w0 = 1.0f - wh;
            e.w1 = wh;
        }
        tab[j] = e;
    }
#pragma unroll
    for (int q = 0; q < 12; q++) pc[q][i] = 0.0f;
    float e = 0.0f;
    int L = 0;
    float a0 = 0.0f, a1 = 0.0f;
    auto flush = [&]() {  // semitone bin L is final: fold it into chroma and energy
        if (a0 > 0.0f) {
            int cls = (P.log_off + L) % 12;
            if (cls < 0) cls += 12;
            pc[cls][i] += a0;
        }
        e += a0 * a0;
        a0 = a1;
        a1 = 0.0f;
        L++;
    };
    const int sub = i / CW, jj = i % CW;
    const int64_t rows = F - f0 < HP_FRAMES ? F - f0 : HP_FRAMES;
    constexpr int NLD = CW;
    constexpr int RSTEP = HP_FRAMES / CW;
    const float* rowp = mags + (g0 + (uint64_t)f0 + (uint64_t)sub) * (uint64_t)P.stride + jj;
    const uint64_t rstride = (uint64_t)RSTEP * (uint64_t)P.stride;
    float nx[NLD];
    auto load_chunk = [&](int c0) {
        const bool col_ok = c0 + jj < P.B;
#pragma unroll
        for (int u = 0; u < NLD; u++)
            nx[u] = (sub + u * RSTEP < rows && col_ok) ? rowp[(uint64_t)u * rstride + c0] : 0.0f;
    };
    // MODE 1 reads only the log-frequency band; MODE 0 also folds the energy over every bin
    const int cend = MODE == 0 ? P.B : (P.hi + 1 < P.B ? P.hi + 1 : P.B);
    const int cbeg = MODE == 0 ? 0 : (P.lo / CW) * CW;
    load_chunk(cbeg);
    for (int c0 = cbeg; c0 < cend; c0 += CW) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < NLD; u++) tile[sub + u * RSTEP][jj] = nx[u];
        __syncthreads();
        if (c0 + CW < cend) load_chunk(c0 + CW);
        if (!valid) continue;
        const int cw = cend - c0 < CW ? cend - c0 : CW;
        for (int j = 0; j < cw; j++) {
            const int b = c0 + j;
            const float m = tile[i][j];
            if (MODE == 0) {
                e += m * m;
                if (b >= P.lo && b <= P.hi) {
                    const ChromaBin& t = tab[b - P.lo];
                    const float mag = sd_powf_ool(sd_maxf(m, 0.0f), 0.6f);
                    if (P.soft) {
                        const int p0 = t.a;
                        pc[p0 == 0 ? 11 : p0 - 1][i] += mag * t.w0;
                        pc[p0][i] += mag * t.w1;
                        pc[p0 == 11 ? 0 : p0 + 1][i] += mag * t.w2;
                    } else {
                        pc[t.a][i] += mag;
                    }
                }
            } else {
                if (b >= P.lo && b <= P.hi && m > 0.0f) {
                    const ChromaBin& t = tab[b - P.lo];
                    if (t.a >= 0) {
                        while (L < t.a) flush();
                        a0 += m * t.w0;
                        if (t.b != t.a) a1 += m * t.w1;
                    }
                }
            }
        }
    }
    if (!valid) return;
    if (MODE == 1)
        while (L < P.n_log) flush();
    float nsq = 0.0f;
#pragma unroll
    for (int q = 0; q < 12; q++) nsq += pc[q][i] * pc[q][i];
    const float norm = __builtin_sqrtf(nsq);
    const uint64_t g = g0 + (uint64_t)f;
#pragma unroll
    for (int q = 0; q < 12; q++) {
        float v = pc[q][i];
        if (norm > EPS) v /= norm;
        chroma[g * 12 + q] = v;
    }
    energy[g] = e;
}

// ---------------------------------------------------------------------------------------------
// k_hpcp_x: frame_to_hpcp_tuned_band with the track's tuning offset, optional whitening (WH) and
// the optional bass band (a second top-K list over its own bins; extractor.rs:1154-1244).
// Whitening (extractor.rs:574-596) streams with the bin walk: prefix[b + 1] is known after bin b,
// so whitened[b - half] (window [b - 2 half, b]) is final then; the prefix ring holds the last
// 2 half + 2 prefixes and the raw ring the last half + 1 magnitudes, per thread, in LDS.
// Peak candidates are tested on the (whitened) score stream; the harmonic weights use the raw
// magnitude of each peak bin (re-read from HBM, K loads per frame) and are evaluated per peak
// (the tuning offset moves every pitch class: no shared table).
__device__ inline void hpcp_accumulate(float (*pc)[HP_FRAMES], int i, int bin, float w0, float fres, float fmin,
                                       float fmax, int hmax, float decay, float tuning, float sigma) {
    const float f0 = (float)bin * fres;
    if (f0 <= 0.0f || w0 <= 0.0f) return;
    float dpow = 1.0f;  // decay^(h-1) by __powisf2's square-and-multiply (decay.powi(h - 1))
    for (int h = 1; h <= hmax; h++) {
        const float fh = f0 * (float)h;
        if (fh > fmax) break;
        int e = h - 1;
        float a = decay, r = 1.0f;
        while (true) {
            if (e & 1) r *= a;
            e /= 2;
            if (e == 0) break;
            a *= a;
        }
        dpow = r;
        if (fh < fmin) continue;
        const float semitone = 12.0f * sd_log2f(fh / 440.0f) + 57.0f - tuning;
        const float hw = dpow / (float)h;
        const float contrib = w0 * hw;
        const float spc = sd_rem_euclid_f(semitone, 12.0f);
        const float ppc = sd_rem_euclid_f(sd_roundf(spc), 12.0f);
        const int32_t primary = sd_f2i32(ppc);
        for (int o = -1; o <= 1; o++) {
            const int tc = (((primary + o) % 12) + 12) % 12;
            float dist = sd_absf(spc - (float)tc);
            dist = sd_minf(dist, 12.0f - dist);
            const float sg = sd_maxf(sigma, 1e-6f);
            pc[tc][i] += contrib * sd_expf(-dist * dist / (2.0f * sg * sg));
        }
    }
}

template <int KCAP, int KB>
__device__ __forceinline__ void topk_insert(float (&pm)[KCAP], int (&pb)[KCAP], float& thr, float v, int vb) {
    if (!(v > thr)) return;
    // the descending list's insertion as in HpcpFrame::walk (k_key.hip): gt[q] = v > pm[q] turns
    // true once; slots are updated from the tail in place
    bool gt[KCAP];
#pragma unroll
    for (int q = 0; q < KCAP; q++) gt[q] = v > pm[q];
#pragma unroll
    for (int q = KCAP - 1; q >= 1; q--) {
        // magnitudes: the median of {pm[q], v, pm[q-1]} (the list is descending; v > thr is a number)
        const int nbv = gt[q - 1] ? pb[q - 1] : vb;
        pm[q] = __builtin_amdgcn_fmed3f(pm[q], v, pm[q - 1]);
        pb[q] = gt[q] ? nbv : pb[q];
    }
    pm[0] = gt[0] ? v : pm[0];
    pb[0] = gt[0] ? vb : pb[0];
    thr = pm[KCAP - 1];
}

template <int KCAP, bool WH, bool BASS>
__global__ __launch_bounds__(HP_FRAMES) void k_hpcp_x(const float* __restrict__ mags,
                                                      const uint64_t* __restrict__ frame_pfx,
                                                      const uint64_t* __restrict__ tile_pfx,
                                                      const int* __restrict__ tracks, int n_items, HpcpXParams P,
                                                      const float* __restrict__ tuning, float* __restrict__ chroma,
                                                      float* __restrict__ energy) {
    extern __shared__ float xlds[];  // WH: prefix ring [RP][HP_FRAMES], raw ring [RX][HP_FRAMES]
    __shared__ float tile[HP_FRAMES][CW + 1];
    __shared__ float pcb[BASS ? 12 : 1][HP_FRAMES];
    const uint64_t gb = blockIdx.x;
    const int it = find_track(tile_pfx, n_items, gb);
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[it]) * HP_FRAMES;
    const int i = threadIdx.x;
    const int64_t f = f0 + i;
    const bool valid = f < F;
    const uint64_t g0 = frame_pfx[trk];
    const float tu = tuning ? tuning[it] : 0.0f;
    float e = 0.0f, m1 = 0.0f, m2 = 0.0f;  // score stream: m1 = s[c], m2 = s[c - 1]
    float pm[KCAP], qm[BASS ? 12 : 1];
    int pb[KCAP], qb[BASS ? 12 : 1];
#pragma unroll
    for (int q = 0; q < KCAP; q++) pm[q] = -1.0f, pb[q] = 0;
#pragma unroll
    for (int q = 0; q < (BASS ? 12 : 1); q++) qm[q] = -1.0f, qb[q] = 0;
    float thr = -1.0f, qthr = -1.0f;
    // whitening state
    float* ringP = xlds + i;
    float* ringX = xlds + (size_t)P.rp * HP_FRAMES + i;
    const int half = P.half;
    float prefix = 0.0f;
    if (WH) ringP[0] = 0.0f;
    int c = -1;  // index of the next score-stream element
    auto feed = [&](float s) {  // s = score[c + 1]; tests candidate c
        const int cc = c;
        if (cc >= 1 && !(m1 <= m2 || m1 < s)) {
            if (cc >= P.pk_lo && cc <= P.pk_hi) topk_insert<KCAP, KCAP>(pm, pb, thr, m1, cc);
            if (BASS && cc >= P.bk_lo && cc <= P.bk_hi) topk_insert<(BASS ? 12 : 1), 12>(qm, qb, qthr, m1, cc);
        }
        m2 = m1;
        m1 = s;
        c++;
    };
    auto white_at = [&](int wi, int r) {  // whitened[wi] with window [max(wi - half, 0), r]
        const int l = wi >= half ? wi - half : 0;
        const float denom = (float)(r + 1 - l);
        const float mean = (ringP[((r + 1) & P.rp_mask) * HP_FRAMES] - ringP[(l & P.rp_mask) * HP_FRAMES]) /
                           sd_maxf(denom, 1.0f);
        const float v = sd_maxf(ringX[(wi & P.rx_mask) * HP_FRAMES], 0.0f) / (mean + 1e-12f);
        return sd_minf(v, 20.0f);
    };
    const int sub = i / CW, jj = i % CW;
    const int64_t rows = F - f0 < HP_FRAMES ? F - f0 : HP_FRAMES;
    constexpr int NLD = CW;
    constexpr int RSTEP = HP_FRAMES / CW;
    const float* rowp = mags + (g0 + (uint64_t)f0 + (uint64_t)sub) * (uint64_t)P.stride + jj;
    const uint64_t rstride = (uint64_t)RSTEP * (uint64_t)P.stride;
    float nx[NLD];
    auto load_chunk = [&](int c0) {
        const bool col_ok = c0 + jj < P.B;
#pragma unroll
        for (int u = 0; u < NLD; u++)
            nx[u] = (sub + u * RSTEP < rows && col_ok) ? rowp[(uint64_t)u * rstride + c0] : 0.0f;
    };
    load_chunk(0);
    for (int c0 = 0; c0 < P.B; c0 += CW) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < NLD; u++) tile[sub + u * RSTEP][jj] = nx[u];
        __syncthreads();
        if (c0 + CW < P.B) load_chunk(c0 + CW);
        if (!valid) continue;
        const int cw = P.B - c0 < CW ? P.B - c0 : CW;
        for (int j = 0; j < cw; j++) {
            const int b = c0 + j;
            const float m = tile[i][j];
            e += m * m;
            if (WH) {
                prefix = prefix + sd_maxf(m, 0.0f);
                ringP[((b + 1) & P.rp_mask) * HP_FRAMES] = prefix;
                ringX[(b & P.rx_mask) * HP_FRAMES] = m;
                if (b >= half) feed(white_at(b - half, b));
            } else {
                feed(m);
            }
        }
    }
    // pitch-class accumulators reuse the staging tile
    __syncthreads();
    float(*pc)[HP_FRAMES] = reinterpret_cast<float(*)[HP_FRAMES]>(&tile[0][0]);
    if (!valid) return;
    if (WH)
        for (int wi = P.B - half > 0 ? P.B - half : 0; wi < P.B; wi++) feed(white_at(wi, P.B - 1));
    // the last bin is never a candidate (bin + 1 < bins)
#pragma unroll
    for (int q = 0; q < 12; q++) pc[q][i] = 0.0f;
    const uint64_t g = g0 + (uint64_t)f;
    const float* rowg = mags + g * (uint64_t)P.stride;
    if (P.main_ok) {
        for (int k = 0; k < KCAP; k++) {
            if (k >= P.K || !(pm[k] > 0.0f)) continue;
            const float raw = WH ? rowg[pb[k]] : pm[k];
            const float w0 = sd_powf_ool(sd_maxf(raw, 0.0f), P.p);
            hpcp_accumulate(pc, i, pb[k], w0, P.fres, P.fmin, P.fmax, P.hmax, P.decay, tu, P.sigma);
        }
    }
    float out[12];
    {
        float nsq = 0.0f;
#pragma unroll
        for (int q = 0; q < 12; q++) nsq += pc[q][i] * pc[q][i];
        const float norm = __builtin_sqrtf(nsq);
#pragma unroll
        for (int q = 0; q < 12; q++) out[q] = norm > EPS ? pc[q][i] / norm : pc[q][i];
    }
    if (BASS) {
#pragma unroll
        for (int q = 0; q < 12; q++) pcb[q][i] = 0.0f;
        if (P.bass_ok) {
            for (int k = 0; k < 12; k++) {
                if (k >= P.KB || !(qm[k] > 0.0f)) continue;
                const float raw = WH ? rowg[qb[k]] : qm[k];
                const float w0 = sd_powf_ool(sd_maxf(raw, 0.0f), P.p);
                hpcp_accumulate(pcb, i, qb[k], w0, P.fres, P.bfmin, P.bfmax, P.hmax, P.decay, tu, P.sigma);
            }
        }
        float nsq = 0.0f;
#pragma unroll
        for (int q = 0; q < 12; q++) nsq += pcb[q][i] * pcb[q][i];
        const float norm = __builtin_sqrtf(nsq);
        float bl[12];
        float n2 = 0.0f;
#pragma unroll
        for (int q = 0; q < 12; q++) {
            const float bq = norm > EPS ? pcb[q][i] / norm : pcb[q][i];
            bl[q] = (1.0f - P.bw) * out[q] + P.bw * bq;
            n2 += bl[q] * bl[q];
        }
        const float nb = __builtin_sqrtf(n2);
#pragma unroll
        for (int q = 0; q < 12; q++) out[q] = nb > 1e-10f ? bl[q] / nb : bl[q];
    }
#pragma unroll
    for (int q = 0; q < 12; q++) chroma[g * 12 + q] = out[q];
    energy[g] = e;
}

// ---------------------------------------------------------------------------------------------
// k_beat_sync: one workgroup per track, one thread per beat interval [beats[j], beats[j+1]).
// Frame times t_f = f * (hop / sr) are non-decreasing in f, so the frames of an interval are
// the contiguous range [first t_f >= start, first t_f >= end); their chroma rows are summed in
// frame order (extractor.rs:871-926).
__device__ inline int64_t first_time_ge(float x, float fd, int64_t F) {
    int64_t lo = 0, hi = F;  // first f in [0, F] with (float)f * fd >= x
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((float)mid * fd >= x)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}
__global__ __launch_bounds__(256) void k_beat_sync(const int* __restrict__ tracks, const uint64_t* __restrict__ frame_pfx,
                                                   const float* __restrict__ fchroma, const float* __restrict__ fenergy,
                                                   const float* __restrict__ beats, const uint64_t* __restrict__ beat_off,
                                                   const uint64_t* __restrict__ row_pfx, float fd,
                                                   float* __restrict__ chroma, float* __restrict__ energy) {
    const int it = blockIdx.x;
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const float* fc = fchroma + frame_pfx[trk] * 12;
    const float* fe = fenergy + frame_pfx[trk];
    const float* bt = beats + beat_off[it];
    const uint64_t r0 = row_pfx[it];
    const int64_t NB = (int64_t)(row_pfx[it + 1] - r0);
    for (int64_t j = threadIdx.x; j < NB; j += blockDim.x) {
        const float bs = bt[j], be = bt[j + 1];
        const int64_t a = first_time_ge(bs, fd, F);
        const int64_t z = first_time_ge(be, fd, F);
        float avg[12];
#pragma unroll
        for (int q = 0; q < 12; q++) avg[q] = 0.0f;
        float en = 0.0f;
        for (int64_t k = a; k < z; k++) {
#pragma unroll
            for (int q = 0; q < 12; q++) avg[q] += fc[k * 12 + q];
            en += fe[k];
        }
        float* o = chroma + (r0 + (uint64_t)j) * 12;
        if (z > a) {
            const float n = (float)(z - a);
            float nsq = 0.0f;
#pragma unroll
            for (int q = 0; q < 12; q++) {
                avg[q] /= n;
                nsq += avg[q] * avg[q];
            }
            const float norm = __builtin_sqrtf(nsq);
            if (norm > EPS)
#pragma unroll
                for (int q = 0; q < 12; q++) avg[q] /= norm;
        } else {
            en = 0.0f;
        }
#pragma unroll
        for (int q = 0; q < 12; q++) o[q] = avg[q];
        energy[r0 + (uint64_t)j] = en;
    }
}

// ---------------------------------------------------------------------------------------------
// Key HPSS median mask (extractor.rs:1369-1501).  k_key_hpss_mask: for every downsampled frame k
// (every `step`-th frame) and band bin b, the median over time (ds frames k +- tm) and over
// frequency (bins b +- fm) of the sanitised magnitudes, and the soft mask h^p / (h^p + p^p + eps).
// A workgroup owns KH_TK ds frames x 64 bins; the tile plus its halo is staged in LDS, and each
// median is a rank selection over the window held in registers (out-of-range slots are +inf, so
// they rank last and the order statistic len/2 of the real values is unchanged).
constexpr int KH_TK = 16, KH_MAXM = 16, KH_COLS = 64;
__device__ __forceinline__ float kh_san(float x) { return sd_isfinite_f(x) ? sd_maxf(x, 0.0f) : 0.0f; }

template <int W>
__device__ __forceinline__ float rank_select(const float (&v)[W], int mid) {
    float med = 0.0f;
#pragma unroll
    for (int j = 0; j < W; j++) {
        int lt = 0, le = 0;
#pragma unroll
        for (int q = 0; q < W; q++) {
            lt += v[q] < v[j];
            le += v[q] <= v[j];
        }
        if (lt <= mid && mid < le) med = v[j];
    }
    return med;
}

template <int M>  // M: compile-time window half width bound (== the margins when FIXED)
__global__ __launch_bounds__(256) void k_key_hpss_mask(const float* __restrict__ mags,
                                                       const uint64_t* __restrict__ frame_pfx,
                                                       const uint64_t* __restrict__ tile_pfx,
                                                       const uint64_t* __restrict__ mask_off,
                                                       const int* __restrict__ tracks, int n_items, KeyHpssParams P,
                                                       float* __restrict__ mask) {
    constexpr int W = 2 * M + 1;
    __shared__ float tl[KH_TK + 2 * KH_MAXM][KH_COLS + 2 * KH_MAXM + 1];
    const uint64_t gb = blockIdx.x;
    const int it = find_track(tile_pfx, n_items, gb);
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t nds = F > 0 ? (F + P.step - 1) / P.step : 1;
    const int64_t nbt = (P.nb + KH_COLS - 1) / KH_COLS;
    const int64_t lt_ = (int64_t)(gb - tile_pfx[it]);
    const int64_t k0 = (lt_ / nbt) * KH_TK;
    const int b0 = (int)(lt_ % nbt) * KH_COLS;
    const float* base = mags + frame_pfx[trk] * (uint64_t)P.stride + P.bin0;
    const int tm = P.tm, fm = P.fm;
    const int rows = KH_TK + 2 * tm, cols = KH_COLS + 2 * fm;
    const float INF = __builtin_inff();
    for (int e = threadIdx.x; e < rows * cols; e += 256) {
        const int r = e / cols, c = e % cols;
        const int64_t k = k0 - tm + r;
        const int b = b0 - fm + c;
        float v = INF;
        if (k >= 0 && k < nds && b >= 0 && b < P.nb) v = kh_san(base[(uint64_t)(k * P.step) * (uint64_t)P.stride + b]);
        tl[r][c] = v;
    }
    __syncthreads();
    const int c = threadIdx.x % KH_COLS, q0 = threadIdx.x / KH_COLS;
    const int b = b0 + c;
    if (b >= P.nb) return;
    float* mo = mask + mask_off[it];
    for (int kk = q0; kk < KH_TK; kk += 256 / KH_COLS) {
        const int64_t k = k0 + kk;
        if (k >= nds) break;
        float v[W];
#pragma unroll
        for (int o = 0; o < W; o++) {
            const int d = o - M;
            v[o] = (d >= -tm && d <= tm) ? tl[kk + tm + d][c + fm] : INF;
        }
        const int64_t ts = k >= tm ? k - tm : 0, te = k + tm + 1 < nds ? k + tm + 1 : nds;
        const float h = rank_select<W>(v, (int)((te - ts) / 2));
#pragma unroll
        for (int o = 0; o < W; o++) {
            const int d = o - M;
            v[o] = (d >= -fm && d <= fm) ? tl[kk + tm][c + fm + d] : INF;
        }
        const int bs = b >= fm ? b - fm : 0, be = b + fm + 1 < P.nb ? b + fm + 1 : P.nb;
        const float pe = rank_select<W>(v, (be - bs) / 2);
        const float hh = sd_maxf(h, 0.0f), pp = sd_maxf(pe, 0.0f);
        const float hp = sd_powf(hh, P.p), ppw = sd_powf(pp, P.p);
        mo[(uint64_t)k * (uint64_t)P.nb + (uint64_t)b] = hp / (hp + ppw + 1e-12f);
    }
}

// Applies the downsampled mask to every frame in place: band bins -> sanitised x * mask, every
// other bin -> 0 (the reference's output rows start as zeros).  KH_FR frames per workgroup.
constexpr int KH_FR = 8;
__global__ __launch_bounds__(256) void k_key_hpss_apply(float* __restrict__ mags, const uint64_t* __restrict__ frame_pfx,
                                                        const uint64_t* __restrict__ tile_pfx,
                                                        const uint64_t* __restrict__ mask_off,
                                                        const int* __restrict__ tracks, int n_items, KeyHpssParams P,
                                                        const float* __restrict__ mask) {
    const uint64_t gb = blockIdx.x;
    const int it = find_track(tile_pfx, n_items, gb);
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t nds = (F + P.step - 1) / P.step;
    const int64_t t0 = (int64_t)(gb - tile_pfx[it]) * KH_FR;
    const float* mo = mask + mask_off[it];
    for (int64_t t = t0; t < t0 + KH_FR && t < F; t++) {
        float* row = mags + (frame_pfx[trk] + (uint64_t)t) * (uint64_t)P.stride;
        int64_t k = t / P.step;
        if (k > nds - 1) k = nds - 1;
        const float* mk = mo + (uint64_t)k * (uint64_t)P.nb;
        for (int b = threadIdx.x; b < P.B; b += 256) {
            const int j = b - P.bin0;
            row[b] = (j >= 0 && j < P.nb) ? kh_san(row[b]) * mk[j] : 0.0f;
        }
    }
}

// ---- launchers ----
void launch_tuning(const float* mags, const uint64_t* frame_pfx, const int* tracks, int n_items, const TuningParams& P,
                   float* out, hipStream_t st) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_tuning, dim3(n_items), dim3(TU_T), 0, st, mags, frame_pfx, tracks, P, out);
}
void launch_chroma(int mode, const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                   int n_items, uint64_t n_tiles, const ChromaParams& P, const float* tuning, float* chroma,
                   float* energy, hipStream_t st) {
    if (n_tiles == 0) return;
    const size_t lds = (size_t)(P.hi - P.lo + 1) * sizeof(ChromaBin);
    if (mode == 0)
        hipLaunchKernelGGL(k_chroma<0>, dim3((unsigned)n_tiles), dim3(HP_FRAMES), lds, st, mags, frame_pfx, tile_pfx,
                           tracks, n_items, P, tuning, chroma, energy);
    else
        hipLaunchKernelGGL(k_chroma<1>, dim3((unsigned)n_tiles), dim3(HP_FRAMES), lds, st, mags, frame_pfx, tile_pfx,
                           tracks, n_items, P, tuning, chroma, energy);
}
template <int KCAP>
static void hpcp_x_dispatch(bool wh, bool bass, dim3 g, size_t lds, hipStream_t st, const float* mags,
                            const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks, int n_items,
                            const HpcpXParams& P, const float* tuning, float* chroma, float* energy) {
    const dim3 b(HP_FRAMES);
    if (wh && bass)
        hipLaunchKernelGGL((k_hpcp_x<KCAP, true, true>), g, b, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items, P,
                           tuning, chroma, energy);
    else if (wh)
        hipLaunchKernelGGL((k_hpcp_x<KCAP, true, false>), g, b, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items, P,
                           tuning, chroma, energy);
    else if (bass)
        hipLaunchKernelGGL((k_hpcp_x<KCAP, false, true>), g, b, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items, P,
                           tuning, chroma, energy);
    else
        hipLaunchKernelGGL((k_hpcp_x<KCAP, false, false>), g, b, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items,
                           P, tuning, chroma, energy);
}
void launch_hpcp_x(const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                   int n_items, uint64_t n_tiles, const HpcpXParams& P, const float* tuning, float* chroma,
                   float* energy, hipStream_t st) {
    if (n_tiles == 0) return;
    const bool wh = P.half > 0;
    const size_t lds = wh ? (size_t)(P.rp + P.rx) * HP_FRAMES * sizeof(float) : 0;
    const dim3 g((unsigned)n_tiles);
    if (P.K <= 8)
        hpcp_x_dispatch<8>(wh, P.bass, g, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, tuning, chroma, energy);
    else if (P.K <= 16)
        hpcp_x_dispatch<16>(wh, P.bass, g, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, tuning, chroma,
                            energy);
    else if (P.K <= 24)
        hpcp_x_dispatch<24>(wh, P.bass, g, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, tuning, chroma,
                            energy);
    else
        hpcp_x_dispatch<HP_KMAX>(wh, P.bass, g, lds, st, mags, frame_pfx, tile_pfx, tracks, n_items, P, tuning, chroma,
                                 energy);
}
void launch_key_hpss(float* mags, const uint64_t* frame_pfx, const uint64_t* mtile_pfx, uint64_t n_mtiles,
                     const uint64_t* atile_pfx, uint64_t n_atiles, const uint64_t* mask_off, const int* tracks,
                     int n_items, const KeyHpssParams& P, float* mask, hipStream_t st) {
    if (n_items == 0) return;
    if (P.tm <= 8 && P.fm <= 8)
        hipLaunchKernelGGL(k_key_hpss_mask<8>, dim3((unsigned)n_mtiles), dim3(256), 0, st, mags, frame_pfx, mtile_pfx,
                           mask_off, tracks, n_items, P, mask);
    else
        hipLaunchKernelGGL(k_key_hpss_mask<KH_MAXM>, dim3((unsigned)n_mtiles), dim3(256), 0, st, mags, frame_pfx,
                           mtile_pfx, mask_off, tracks, n_items, P, mask);
    hipLaunchKernelGGL(k_key_hpss_apply, dim3((unsigned)n_atiles), dim3(256), 0, st, mags, frame_pfx, atile_pfx,
                       mask_off, tracks, n_items, P, mask);
}
void launch_beat_sync(const int* tracks, int n_items, const uint64_t* frame_pfx, const float* fchroma,
                      const float* fenergy, const float* beats, const uint64_t* beat_off, const uint64_t* row_pfx,
                      float fd, float* chroma, float* energy, hipStream_t st) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_beat_sync, dim3(n_items), dim3(256), 0, st, tracks, frame_pfx, fchroma, fenergy, beats,
                       beat_off, row_pfx, fd, chroma, energy);
}

}  // namespace sdsp
