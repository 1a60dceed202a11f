// k_key.hip — key detection path (reference src/lib.rs:961-1559):
//
//   k_mask      harmonic_spectrogram_time_mask + smooth_spectrogram_time  chroma/extractor.rs:1246-1349
//   k_hpcp      HPCP chroma + frame energies                              extractor.rs:529-680, 1097-1150
//   k_key_vote  median smoothing, frame weights, segment voting,         smoothing.rs:37-94, src/lib.rs:1211-1436,
//               detect_key_weighted, key clarity                          key/detector.rs:68-313, key_clarity.rs:51-93
//
// k_mask: one thread per (track, bin) streams the track's frames in order, carrying the
// reference's sequential per-bin f32 prefix sum (prefix[t+1] = prefix[t] + x) in a 2M+2-slot
// ring in LDS; adjacent lanes touch adjacent bins of the same frame, so every HBM access is a
// coalesced 1 KB row segment.  The mask is applied in place.
#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdsp {

constexpr int MASK_T = 256;
constexpr int MASK_RING_MAX = 64;

__global__ __launch_bounds__(MASK_T) void k_mask(float* __restrict__ mags, int stride, int B,
                                                  const uint64_t* __restrict__ frame_pfx, const int* __restrict__ tracks,
                                                  int blocks_per_track, int margin, float power) {
    __shared__ float ring[MASK_RING_MAX][MASK_T];
    const int it = blockIdx.x / blocks_per_track;
    const int trk = tracks[it];
    const int b = (blockIdx.x % blocks_per_track) * MASK_T + threadIdx.x;
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    if (b >= B || F <= 0) return;
    float* col = mags + frame_pfx[trk] * (uint64_t)stride + b;
    const int R = 2 * margin + 2;
    const float p = sd_maxf(power, 1.0f);
    const float eps = 1e-12f;
    float* rg = &ring[0][threadIdx.x];
    rg[0] = 0.0f;
    float prev = 0.0f;
    for (int64_t tin = 0; tin < F + margin; tin++) {
        if (tin < F) {
            prev = prev + col[tin * stride];
            rg[((tin + 1) % R) * MASK_T] = prev;
        }
        const int64_t t = tin - margin;
        if (t < 0) continue;
        if (t >= F) break;
        const int64_t st = t >= margin ? t - margin : 0;
        const int64_t en = t + margin + 1 < F ? t + margin + 1 : F;
        const float denom = (float)(en - st > 1 ? en - st : 1);
        const float xr = col[t * stride];
        // margin 0: smooth_spectrogram_time returns its input unchanged (extractor.rs:1250-1252)
        const float hm = margin == 0 ? xr : (rg[(en % R) * MASK_T] - rg[(st % R) * MASK_T]) / denom;
        const float x = sd_maxf(xr, 0.0f);
        const float h = sd_maxf(hm, 0.0f);
        const float r = sd_maxf(x - h, 0.0f);
        const float hp = sd_powf(h, p);
        const float rp = sd_powf(r, p);
        const float m = hp / (hp + rp + eps);
        col[t * stride] = x * m;
    }
}

// ----------------------------------------------------------------------------------------
constexpr int HP_T = 64;     // frames per workgroup (one per thread)
constexpr int HP_CW = 64;    // bins per staged chunk

__global__ __launch_bounds__(HP_T) void k_hpcp(const float* __restrict__ mags, const uint64_t* __restrict__ frame_pfx,
                                               const uint64_t* __restrict__ tile_pfx, const int* __restrict__ tracks,
                                               int n_items, HpcpParams P, const HarmEntry* __restrict__ harm,
                                               float* __restrict__ chroma, float* __restrict__ energy) {
    __shared__ float tile[HP_T][HP_CW + 1];
    __shared__ float pk_m[HP_KMAX][HP_T];
    __shared__ int pk_b[HP_KMAX][HP_T];
    __shared__ float pc[12][HP_T];
    const uint64_t gb = blockIdx.x;
    const int it = find_track(tile_pfx, n_items, gb);
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[it]) * HP_T;
    const int i = threadIdx.x;
    const int64_t f = f0 + i;
    const bool valid = f < F;
    const uint64_t g0 = frame_pfx[trk];
    float e = 0.0f, m1 = 0.0f, m2 = 0.0f;  // m1 = m[b-1], m2 = m[b-2]
    int npk = 0;
    for (int c0 = 0; c0 < P.B; c0 += HP_CW) {
        __syncthreads();
        const int cw = P.B - c0 < HP_CW ? P.B - c0 : HP_CW;
        for (int idx = i; idx < HP_T * HP_CW; idx += HP_T) {
            const int r = idx / HP_CW, j = idx % HP_CW;
            float v = 0.0f;
            if (f0 + r < F && j < cw) v = mags[(g0 + (uint64_t)(f0 + r)) * (uint64_t)P.stride + c0 + j];
            tile[r][j] = v;
        }
        __syncthreads();
        if (!valid) continue;
        for (int j = 0; j < cw; j++) {
            const int b = c0 + j;
            const float m = tile[i][j];
            e += m * m;
            const int c = b - 1;  // candidate peak bin, needs m[c-1] = m2, m[c] = m1, m[c+1] = m
            if (c >= P.pk_lo && c <= P.pk_hi) {
                if (!(m1 <= m2 || m1 < m)) {
                    // insert (m1, c) keeping (mag desc, bin asc); bins arrive ascending
                    int pos = npk;
                    while (pos > 0 && pk_m[pos - 1][i] < m1) pos--;
                    if (pos < P.K) {
                        const int last = npk < P.K ? npk : P.K - 1;
                        for (int q = last; q > pos; q--) {
                            pk_m[q][i] = pk_m[q - 1][i];
                            pk_b[q][i] = pk_b[q - 1][i];
                        }
                        pk_m[pos][i] = m1;
                        pk_b[pos][i] = c;
                        if (npk < P.K) npk++;
                    }
                }
            }
            m2 = m1;
            m1 = m;
        }
    }
    if (!valid) return;
    for (int q = 0; q < 12; q++) pc[q][i] = 0.0f;
    for (int k = 0; k < npk; k++) {
        const int bin = pk_b[k][i];
        const float w0 = sd_powf(sd_maxf(pk_m[k][i], 0.0f), P.p);
        if (w0 <= 0.0f) continue;
        for (int h = 1; h <= P.hmax; h++) {
            const HarmEntry he = harm[bin * HP_HMAX + (h - 1)];
            if (he.state == 0) break;
            if (he.state == 1) continue;
            const float contrib = w0 * he.hw;
            for (int o = 0; o < 3; o++) pc[he.tc[o]][i] += contrib * he.wt[o];
        }
    }
    float nsq = 0.0f;
    for (int q = 0; q < 12; q++) nsq += pc[q][i] * pc[q][i];
    const float norm = __builtin_sqrtf(nsq);
    const uint64_t g = g0 + (uint64_t)f;
    for (int q = 0; q < 12; q++) {
        float v = pc[q][i];
        if (norm > EPS) v /= norm;
        chroma[g * 12 + q] = v;
    }
    energy[g] = e;
}

// ----------------------------------------------------------------------------------------
__device__ void key_from_raw(const float raw[24], float sorted[24], int order[24]) {
    float sc[24];
    for (int k = 0; k < 24; k++) sc[k] = raw[k];
    float mM = 0.0f, mm = 0.0f;
    for (int k = 0; k < 12; k++) mM = sd_maxf(mM, sc[k]);
    for (int k = 0; k < 12; k++) mm = sd_maxf(mm, sc[12 + k]);
    if (mM > 1e-9f && mm > 1e-9f) {
        for (int k = 0; k < 12; k++) sc[k] /= mM;
        for (int k = 0; k < 12; k++) sc[12 + k] /= mm;
    }
    int tM = 0, tm = 0;
    for (int k = 1; k < 12; k++)
        if (!(sc[k] < sc[tM])) tM = k;
    for (int k = 1; k < 12; k++)
        if (!(sc[12 + k] < sc[12 + tm])) tm = k;
    const float tMs = sc[tM], tms = sc[12 + tm];
    const int cof_pos[12] = {0, 7, 2, 9, 4, 11, 6, 1, 8, 3, 10, 5};  // position of tonic on the circle
    float rs[24];
    for (int k = 0; k < 24; k++) {
        rs[k] = sc[k];
        const bool major = k < 12;
        const int ref_t = major ? tM : tm;
        const float ref_s = major ? tMs : tms;
        if (ref_s > 1e-9f) {
            const int tp = cof_pos[k % 12], rp = cof_pos[ref_t];
            const int ad = tp > rp ? tp - rp : rp - tp;
            const int dist = ad < 12 - ad ? ad : 12 - ad;
            if (dist <= 2) rs[k] += ref_s * (0.20f * (1.0f - (float)dist * 0.5f));
        }
    }
    for (int k = 0; k < 24; k++) order[k] = k;
    for (int a = 1; a < 24; a++) {  // stable insertion sort, desc
        const int o = order[a];
        int b = a;
        while (b > 0 && rs[order[b - 1]] < rs[o]) {
            order[b] = order[b - 1];
            b--;
        }
        order[b] = o;
    }
    for (int k = 0; k < 24; k++) sorted[k] = rs[order[k]];
}

__device__ float clarity_of(const float* s) {
    const float best = s[0];
    float sum = 0.0f;
    for (int i = 0; i < 24; i++) sum += s[i];
    const float avg = sum / 24.0f;
    float mn = s[0], mx = s[0];
    for (int i = 1; i < 24; i++) {
        if (s[i] < mn) mn = s[i];
        if (!(s[i] < mx)) mx = s[i];
    }
    const float range = mx - mn;
    return range > 1e-10f ? sd_clampf((best - avg) / range, 0.0f, 1.0f) : 0.0f;
}

// cof_pos above maps a tonic to its circle-of-fifths position: the reference searches
// circle_of_fifths = [0,7,2,9,4,11,6,1,8,3,10,5] for the tonic (detector.rs:214-224); that
// array is its own inverse, so position(t) = circle_of_fifths[t].

__global__ __launch_bounds__(256) void k_key_vote(const int* __restrict__ tracks, int n_items,
                                                  const uint64_t* __restrict__ frame_pfx,
                                                  const float* __restrict__ chroma_raw,
                                                  const float* __restrict__ energy, float* __restrict__ chroma_s,
                                                  float* __restrict__ weights, float* __restrict__ seg_scratch,
                                                  const uint64_t* __restrict__ seg_off, const float* __restrict__ tmpl,
                                                  KeyParams P, KeyOut* __restrict__ out) {
    __shared__ int hist[256];
    __shared__ int misc[4];
    __shared__ int redi[8];
    __shared__ float acc[24];
    __shared__ int use_w_s, used_s;
    __shared__ float tpl[24][12];
    const int it = blockIdx.x;
    const int trk = tracks[it];
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const uint64_t g0 = frame_pfx[trk];
    const float* cr = chroma_raw + g0 * 12;
    float* cs = chroma_s + g0 * 12;
    float* w = weights + g0;
    const float* en = energy + g0;
    for (int k = threadIdx.x; k < 288; k += blockDim.x) tpl[k / 12][k % 12] = tmpl[k];
    if (F <= 0) {
        if (threadIdx.x == 0) out[trk] = KeyOut{0, 0, 0.0f, 0.0f, 0, 0, 0};
        return;
    }
    // median smoothing, window 5 (src/lib.rs:1211-1213 -> smoothing.rs:37-94)
    for (int64_t q = threadIdx.x; q < F * 12; q += blockDim.x) {
        const int64_t f = q / 12;
        const int s = (int)(q % 12);
        if (F > 5) {
            float v[5];
            int n = 0;
            for (int o = -2; o <= 2; o++) {
                const int64_t fi = f + o;
                if (fi >= 0 && fi < F) v[n++] = cr[fi * 12 + s];
            }
            for (int a = 1; a < n; a++) {
                const float x = v[a];
                int b = a;
                while (b > 0 && x < v[b - 1]) {
                    v[b] = v[b - 1];
                    b--;
                }
                v[b] = x;
            }
            cs[q] = v[n / 2];
        } else {
            cs[q] = cr[q];
        }
    }
    __syncthreads();
    // frame weights (src/lib.rs:1236-1287)
    if (P.weighting) {
        const float med = sd_maxf(block_select_kth(en, (int)F, (int)(F / 2), hist, misc), 1e-12f);
        const float ln12 = sd_logf(12.0f);
        int used_local = 0;
        for (int64_t f = threadIdx.x; f < F; f += blockDim.x) {
            const float* ch = cs + f * 12;
            float sum = 0.0f;
            for (int k = 0; k < 12; k++) sum += ch[k];
            float tonal = 0.0f;
            if (!(sum <= 1e-12f)) {
                float ent = 0.0f;
                for (int k = 0; k < 12; k++) {
                    const float p = ch[k] / sum;
                    if (p > 1e-12f) ent -= p * sd_logf(p);
                }
                tonal = sd_clampf(1.0f - (ent / ln12), 0.0f, 1.0f);
            }
            if (tonal < P.min_tonal) tonal = 0.0f;
            const float e_norm = sd_maxf(en[f] / med, 0.0f);
            const float wt = sd_powf(tonal, sd_maxf(P.tonal_pow, 0.0f));
            const float we = sd_powf(e_norm, sd_maxf(P.energy_pow, 0.0f));
            const float ww = sd_maxf(wt * we, 0.0f);
            w[f] = ww;
            used_local += ww > 0.0f;
        }
        const int used = block_sum_i(used_local, redi);
        __syncthreads();
        if (threadIdx.x == 0) {
            float sw = 0.0f;
            for (int64_t f = 0; f < F; f++) sw += w[f];
            use_w_s = !(sw <= 1e-12f || used < 10);
        }
    } else if (threadIdx.x == 0) {
        use_w_s = 0;
    }
    __syncthreads();
    const bool use_w = use_w_s;
    auto wsd = [&](int64_t f0, int64_t n, int key) {  // weighted_sum_dot, detector.rs:984-1001
        float a = 0.0f;
        const float* t = tpl[key];
        for (int64_t f = f0; f < f0 + n; f++) {
            const float* c = cs + f * 12;
            if (use_w) {
                const float wt = w[f];
                if (wt > 0.0f) {
                    float d = 0.0f;
                    for (int k = 0; k < 12; k++) d += c[k] * t[k];
                    a += wt * d;
                }
            } else {
                float d = 0.0f;
                for (int k = 0; k < 12; k++) d += c[k] * t[k];
                a += d;
            }
        }
        return a;
    };
    int nseg = 0;
    if (P.seg_voting && F >= P.seg_len) nseg = (int)((F - P.seg_len) / P.seg_hop) + 1;
    float* S = seg_scratch + seg_off[it];  // nseg x (24 sorted scores + 24 order + clarity + used)
    if (nseg > 0) {
        for (int q = threadIdx.x; q < nseg * 24; q += blockDim.x) {
            const int sg = q / 24, k = q % 24;
            S[(size_t)sg * 50 + k] = wsd((int64_t)sg * P.seg_hop, P.seg_len, k);  // raw score
        }
        __syncthreads();
        for (int sg = threadIdx.x; sg < nseg; sg += blockDim.x) {
            float raw[24], sorted[24];
            int order[24];
            for (int k = 0; k < 24; k++) raw[k] = S[(size_t)sg * 50 + k];
            key_from_raw(raw, sorted, order);
            const float cl = clarity_of(sorted);
            for (int k = 0; k < 24; k++) {
                S[(size_t)sg * 50 + k] = sorted[k];
                S[(size_t)sg * 50 + 24 + k] = (float)order[k];
            }
            S[(size_t)sg * 50 + 48] = cl;
            S[(size_t)sg * 50 + 49] = cl >= P.min_clarity ? 1.0f : 0.0f;
        }
        __syncthreads();
        if (threadIdx.x < 24) {
            const int key = threadIdx.x;
            float a = 0.0f;
            for (int sg = 0; sg < nseg; sg++) {
                const float* row = S + (size_t)sg * 50;
                if (row[49] == 0.0f) continue;
                for (int k = 0; k < 24; k++)
                    if ((int)row[24 + k] == key) {
                        a += row[k] * row[48];
                        break;
                    }
            }
            acc[key] = a;
        }
        if (threadIdx.x == 0) {
            int u = 0;
            for (int sg = 0; sg < nseg; sg++) u += S[(size_t)sg * 50 + 49] != 0.0f;
            used_s = u;
        }
        __syncthreads();
    } else if (threadIdx.x == 0) {
        used_s = 0;
    }
    __syncthreads();
    const int used = used_s;
    if (used == 0) {  // whole-slice detect_key_weighted
        if (threadIdx.x < 24) acc[threadIdx.x] = wsd(0, F, threadIdx.x);
        __syncthreads();
        if (threadIdx.x == 0) {
            float raw[24], sorted[24];
            int order[24];
            for (int k = 0; k < 24; k++) raw[k] = acc[k];
            key_from_raw(raw, sorted, order);
            KeyOut r{};
            r.mode = order[0] < 12 ? 0 : 1;
            r.tonic = order[0] % 12;
            r.conf = sorted[0] > 0.0f ? sd_clampf((sorted[0] - sorted[1]) / sorted[0], 0.0f, 1.0f) : 0.0f;
            r.clarity = clarity_of(sorted);
            r.ok = 1;
            r.used_segments = 0;
            r.weights_used = use_w;
            out[trk] = r;
        }
        return;
    }
    if (threadIdx.x == 0) {
        int order[24];
        for (int k = 0; k < 24; k++) order[k] = k;
        for (int a = 1; a < 24; a++) {
            const int o = order[a];
            int b = a;
            while (b > 0 && acc[order[b - 1]] < acc[o]) {
                order[b] = order[b - 1];
                b--;
            }
            order[b] = o;
        }
        float sorted[24];
        for (int k = 0; k < 24; k++) sorted[k] = acc[order[k]];
        KeyOut r{};
        r.mode = order[0] < 12 ? 0 : 1;
        r.tonic = order[0] % 12;
        const float bs = sorted[0], ss = sorted[1];
        r.conf = bs > 0.0f ? sd_clampf((bs - ss) / bs, 0.0f, 1.0f) : 0.0f;
        r.clarity = clarity_of(sorted);
        r.ok = 1;
        r.used_segments = used;
        r.weights_used = use_w;
        out[trk] = r;
    }
}

// ---- launchers ----
void launch_mask(float* mags, int stride, int B, const uint64_t* frame_pfx, const int* tracks, int n_items, int margin,
                 float power, hipStream_t st) {
    if (n_items == 0) return;
    const int bpt = (B + MASK_T - 1) / MASK_T;
    hipLaunchKernelGGL(k_mask, dim3(n_items * bpt), dim3(MASK_T), 0, st, mags, stride, B, frame_pfx, tracks, bpt,
                       margin, power);
}
void launch_hpcp(const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                 int n_items, uint64_t n_tiles, const HpcpParams& P, const HarmEntry* harm, float* chroma,
                 float* energy, hipStream_t st) {
    if (n_tiles == 0) return;
    hipLaunchKernelGGL(k_hpcp, dim3((unsigned)n_tiles), dim3(HP_T), 0, st, mags, frame_pfx, tile_pfx, tracks, n_items,
                       P, harm, chroma, energy);
}
void launch_key_vote(const int* tracks, int n_items, const uint64_t* frame_pfx, const float* chroma_raw,
                     const float* energy, float* chroma_s, float* weights, float* seg_scratch, const uint64_t* seg_off,
                     const float* tmpl, const KeyParams& P, KeyOut* out, hipStream_t st) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_key_vote, dim3(n_items), dim3(256), 0, st, tracks, n_items, frame_pfx, chroma_raw, energy,
                       chroma_s, weights, seg_scratch, seg_off, tmpl, P, out);
}

}  // namespace sdsp
