// k_beat.hip — beat grid, one wavefront per track (reference src/features/beat_tracking/):
//
//   HmmBeatTracker::track_beats   hmm.rs:121-441
//   detect_tempo_variations       tempo_variation.rs:95-227
//   BayesianBeatTracker           bayesian.rs:104-272
//   detect_time_signature         time_signature.rs:90-199
//   generate_beat_grid, downbeats, stability   beat_tracking/mod.rs:108-485
//
// The reference's O(frames x onsets) nearest-onset scans become binary searches over the
// sorted onsets (|o - t| is monotone on each side of t in f32, so the nearest neighbour's
// distance is exactly the reference's minimum).  The 64 lanes of the track's wave split the
// independent work: HMM frames (ordered compaction by ballot), Bayesian candidate tempos
// (one lane each, each likelihood folded sequentially as in the reference), the refined-beat
// sort (bitonic with index tie-break == the reference's stable sort) and the three
// time-signature scores.  Sequential folds (interval means, variances, autocorrelation) stay
// on one lane in the reference's order.  The onsets are staged in LDS when they fit.
// The Viterbi pass is not run: the emission is identical for all five states (hmm.rs:264-294),
// so the extracted beats cannot depend on the path and Viterbi cannot fail.
#include "kernels.hpp"

namespace sdsp {

// first index with a[i] >= x (a ascending)
__device__ inline int lower_bound_f(const float* a, int n, float x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < x)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}
// first index with a[i] > x
__device__ inline int upper_bound_f(const float* a, int n, float x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (!(x < a[mid]))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__device__ inline float nearest_dist(const float* on, int n, float t) {
    const int i = lower_bound_f(on, n, t);
    float md = SD_INF_F;
    if (i < n) md = sd_minf(md, sd_absf(on[i] - t));
    if (i > 0) md = sd_minf(md, sd_absf(on[i - 1] - t));
    return md;
}

// hmm.rs:121-441, all lanes of the wave (uniform arguments); returns the number of beats or
// -1 (Err).  *overflow is set when more than `cap` beats would be emitted.
__device__ int hmm_track(float bpm, const float* on, int n, float* out, int cap, int* overflow) {
    if (bpm <= EPS || bpm > 300.0f) return -1;
    if (n <= 0) return -1;
    const int lane = threadIdx.x & 63;
    const float start = on[0], end = on[n - 1];
    const float interval = 60.0f / bpm;
    const uint64_t nf = sd_f2u64(__builtin_ceilf((end - start) / interval)) + 1;
    const float sigma = 0.05f / 2.0f;
    const float sigma_sq = sigma * sigma;
    int nb = 0;
    for (uint64_t t0 = 0; t0 < nf; t0 += 64) {
        const uint64_t t = t0 + (uint64_t)lane;
        bool keep = false;
        float ft = 0.0f;
        if (t < nf) {
            ft = start + ((float)t * interval);
            const float md = nearest_dist(on, n, ft);
            const float dsq = md * md;
            const float em = sd_expf(-dsq / (2.0f * sigma_sq));
            keep = em > 0.1f;
        }
        const unsigned long long bal = __ballot(keep);
        const int pos = nb + __popcll(bal & ((1ull << lane) - 1ull));
        const int cnt = __popcll(bal);
        if (keep && pos < cap) out[pos] = ft;
        if (nb + cnt > cap) {
            *overflow = 1;
            return cap;
        }
        nb += cnt;
    }
    return nb;
}

// Stable ascending sort of a[0..n) into dst[0..n) (the reference's sort_by(partial_cmp) on NaN-free
// data): bitonic over (value, index) keys in LDS, the index breaking ties.  n <= 2*cap_pow2 slots.
__device__ void wave_sort_stable(const float* a, float* dst, int n, float* kv, int* ki, int npow2) {
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < npow2; i += 64) {
        kv[i] = i < n ? a[i] : SD_INF_F;
        ki[i] = i < n ? i : 0x7fffffff;
    }
    __syncthreads();
    for (int k = 2; k <= npow2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = lane; i < npow2; i += 64) {
                const int l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const float vi = kv[i], vl = kv[l];
                    const int ii = ki[i], il = ki[l];
                    const bool gt = (vi > vl) || (vi == vl && ii > il);
                    if (gt == up) {
                        kv[i] = vl;
                        kv[l] = vi;
                        ki[i] = il;
                        ki[l] = ii;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int i = lane; i < n; i += 64) dst[i] = kv[i];
    __syncthreads();
}

// stable bottom-up merge sort (partial_cmp semantics on NaN-free data)
__device__ void merge_sort_f(float* a, float* tmp, int n) {
    for (int w = 1; w < n; w <<= 1) {
        for (int lo = 0; lo < n; lo += 2 * w) {
            const int mid = lo + w < n ? lo + w : n;
            const int hi = lo + 2 * w < n ? lo + 2 * w : n;
            int i = lo, j = mid, k = lo;
            while (i < mid && j < hi) tmp[k++] = (a[j] < a[i]) ? a[j++] : a[i++];
            while (i < mid) tmp[k++] = a[i++];
            while (j < hi) tmp[k++] = a[j++];
        }
        for (int k = 0; k < n; k++) a[k] = tmp[k];
    }
}

struct SegGen {
    const float* b;
    int n;
    float seg_dur, step, cur, last;
    float nominal;
    bool single;  // the single-segment fallback cases
    int phase;    // 0 = running, 1 = emitted single, 2 = done
};

struct Seg {
    float start, end, bpm;
    bool variable;
};

// Replays detect_tempo_variations (tempo_variation.rs:95-227) one segment at a time.
// Returns false when exhausted.  *err set when the reference returns Err.
__device__ bool seg_next(SegGen& g, Seg* s, bool* any_emitted) {
    const float* b = g.b;
    const int n = g.n;
    if (g.phase == 2) return false;
    if (g.single) {
        if (g.phase == 1) {
            g.phase = 2;
            return false;
        }
        g.phase = 1;
        s->start = n == 0 ? 0.0f : b[0];
        s->end = n == 0 ? 0.0f : b[n - 1];
        s->bpm = g.nominal;
        s->variable = false;
        *any_emitted = true;
        return true;
    }
    while (g.cur < g.last) {
        const float cur = g.cur;
        const float se = sd_minf(cur + g.seg_dur, g.last);
        g.cur += g.step;
        const int i0 = lower_bound_f(b, n, cur);
        const int i1 = upper_bound_f(b, n, se);
        if (i1 - i0 < 3) continue;
        float sum = 0.0f;
        int cnt = 0;
        for (int k = i0 + 1; k < i1; k++) {
            const float d = b[k] - b[k - 1];
            if (d > 0.0f) {
                sum += d;
                cnt++;
            }
        }
        if (cnt == 0) continue;
        const float mean = sum / (float)cnt;
        float vs = 0.0f;
        for (int k = i0 + 1; k < i1; k++) {
            const float d = b[k] - b[k - 1];
            if (d > 0.0f) {
                const float dd = d - mean;
                vs += dd * dd;
            }
        }
        const float var = vs / (float)cnt;
        const float sd = __builtin_sqrtf(var);
        const float cv = mean > EPS ? sd / mean : 0.0f;
        s->start = cur;
        s->end = se;
        s->bpm = mean > EPS ? 60.0f / mean : g.nominal;
        s->variable = cv > 0.15f;
        *any_emitted = true;
        return true;
    }
    // exhausted; if nothing was emitted the reference returns one nominal segment
    if (!*any_emitted) {
        g.single = true;
        g.phase = 1;
        s->start = b[0];
        s->end = b[n - 1];
        s->bpm = g.nominal;
        s->variable = false;
        *any_emitted = true;
        return true;
    }
    g.phase = 2;
    return false;
}

__device__ bool seg_init(SegGen& g, const float* b, int n, float nominal) {
    g.b = b;
    g.n = n;
    g.nominal = nominal;
    g.phase = 0;
    g.single = false;
    if (n < 4) {
        g.single = true;
        return true;
    }
    if (nominal <= EPS) return false;  // Err
    const float total = b[n - 1] - b[0];
    if (total < 2.0f) {
        g.single = true;
        return true;
    }
    g.seg_dur = sd_clampf(total / 4.0f, 4.0f, 8.0f);
    const float overlap = g.seg_dur * 0.5f;
    g.step = g.seg_dur - overlap;
    g.cur = b[0];
    g.last = b[n - 1];
    return true;
}

// bayesian.rs:104-178, all lanes (uniform arguments); returns false on Err.  Lane c
// evaluates the c-th candidate tempo (cb advanced by c sequential +0.5 steps, exactly the
// reference's loop variable) with the likelihood folded over the onsets in order; the winner
// is the first candidate reaching the maximum (the reference's strict `lik > best`).
__device__ bool bayes_update(float* cur_bpm, const float* on, int n, float* out_bpm) {
    if (n <= 0) return false;
    if (*cur_bpm <= EPS || *cur_bpm > 300.0f) return false;
    const int lane = threadIdx.x & 63;
    const float lo = sd_maxf(*cur_bpm - 5.0f, 60.0f), hi = sd_minf(*cur_bpm + 5.0f, 180.0f);
    const float sig_sq = 0.05f * 0.05f;
    float cb = lo;
    for (int k = 0; k < lane; k++) cb += 0.5f;
    float lik = -1.0f;  // lanes past `hi` take no part
    if (cb <= hi) {
        const float bi = 60.0f / cb;
        const float st0 = on[0];
        float ll = 0.0f;
        int32_t valid = 0;
        for (int k = 0; k < n; k++) {
            const float o = on[k];
            const int32_t idx = sd_f2i32(sd_roundf((o - st0) / bi));
            const float et = st0 + ((float)idx * bi);
            const float d = sd_absf(o - et);
            ll += -(d * d) / (2.0f * sig_sq);
            valid++;
        }
        lik = valid == 0 ? 0.0f : sd_expf(ll / (float)valid);
    }
    // (lo >= 60 so the reference's `cb <= EPS -> Err` never fires; with 64 lanes and at most
    // 21 candidates every candidate is covered)
    const float m = wave_max(lik);
    float best_bpm = *cur_bpm;
    if (m > 0.0f) {
        const unsigned long long bal = __ballot(lik == m);
        const int w = __ffsll((long long)bal) - 1;
        best_bpm = __shfl(cb, w, 64);
    }
    *cur_bpm = best_bpm;
    *out_bpm = best_bpm;
    return true;
}

__device__ float score_ts(const float* b, int nb, int bpb, float mean, int n_iv) {
    if (n_iv < bpb) return 0.0f;
    // intervals with d > 0, visited in order; autocorrelation at lag bpb over that list
    // (materialised implicitly: iv(k) = k-th positive difference)
    float acc = 0.0f;
    int32_t cnt = 0;
    // walk two cursors over positive differences
    int ka = 1, kb = 1, seen_b = 0;
    // advance kb to the bpb-th positive interval
    while (seen_b < bpb && kb < nb) {
        if (b[kb] - b[kb - 1] > 0.0f) seen_b++;
        kb++;
    }
    // now kb is one past the (bpb)-th positive interval; iv index of kb's next positive = bpb
    for (int i = 0; i + bpb < n_iv; i++) {
        while (!(b[ka] - b[ka - 1] > 0.0f)) ka++;
        while (!(b[kb] - b[kb - 1] > 0.0f)) kb++;
        const float d = sd_absf((b[ka] - b[ka - 1]) - (b[kb] - b[kb - 1]));
        acc += 1.0f / (1.0f + d / mean);
        cnt++;
        ka++;
        kb++;
    }
    if (cnt == 0) return 0.0f;
    const float ac = acc / (float)cnt;
    float vs = 0.0f;
    for (int k = 1; k < nb; k++) {
        const float d = b[k] - b[k - 1];
        if (d > 0.0f) {
            const float dd = d - mean;
            vs += dd * dd;
        }
    }
    const float var = vs / (float)n_iv;
    const float cv = mean > EPS ? __builtin_sqrtf(var) / mean : 1.0f;
    const float cons = 1.0f / (1.0f + cv);
    return sd_minf(ac * 0.7f + cons * 0.3f, 1.0f);
}

// LDS: 32 KB per one-wave workgroup, so k_beat fits on a CU beside the key stream's STFT.  Every
// list the kernel walks sequentially lives in LDS when it fits (a dependent global load costs
// microseconds on a chip whose HBM the key stream saturates; an LDS load ~100 cycles):
constexpr int BEAT_LDS_ON = 4096;    // onsets (then, after the segment loop, the sort keys)
constexpr int BEAT_LDS_B = 2048;     // HMM beats, when the HMM grid has at most this many frames
constexpr int BEAT_SORT_MAX = 2048;  // LDS bitonic sort capacity (larger: serial merge sort); the
                                     // sorted refined beats stay in LDS
static_assert(BEAT_SORT_MAX * 8 <= BEAT_LDS_ON * 4, "sort keys alias the onset buffer");

__global__ __launch_bounds__(64) void k_beat(const int* __restrict__ tracks, int n_items,
                                             const uint32_t* __restrict__ onsets, const uint64_t* __restrict__ on_off,
                                             const int* __restrict__ on_n, uint32_t sr,
                                             const float* __restrict__ bpm_in, const float* __restrict__ conf_in,
                                             float* __restrict__ scratch, const uint64_t* __restrict__ beat_off,
                                             const int* __restrict__ beat_cap, float* __restrict__ beats,
                                             float* __restrict__ downs, BeatOut* __restrict__ out) {
    SDSP_LATENCY_CRITICAL();
    __shared__ float s_on[BEAT_LDS_ON];
    __shared__ float s_hb[BEAT_LDS_B];
    __shared__ float s_rb[BEAT_SORT_MAX];
    float* const s_kv = s_on;  // the onsets are not read after the segment loop
    int* const s_ki = reinterpret_cast<int*>(s_on + BEAT_SORT_MAX);
    const int it = blockIdx.x;
    const int lane = threadIdx.x;
    const int trk = tracks[it];
    BeatOut r{0, 0, 0.0f, 0};
    const float bpm = bpm_in[trk];
    const int n = on_n[trk];
    const int cap = beat_cap[trk];
    // scratch layout per track: [onsets_s | hmm | refined | tmp], each `cap` floats (cap >= n)
    float* ons = scratch + beat_off[trk] * 4;
    float* hb = ons + cap;
    float* rb = hb + cap;
    float* tmp = rb + cap;
    float* ob = beats + beat_off[trk];
    float* od = downs + beat_off[trk];
    auto finish = [&]() {
        if (lane == 0) out[trk] = r;
    };
    int overflow = 0;
    if (!(bpm > 0.0f && n >= 2)) {  // src/lib.rs:913, 944-957
        finish();
        return;
    }
    if (bpm > 300.0f) {  // generate_beat_grid InvalidInput
        finish();
        return;
    }
    const uint32_t* os = onsets + on_off[trk];
    float* onp = n <= BEAT_LDS_ON ? s_on : ons;
    for (int k = lane; k < n; k += 64) onp[k] = (float)os[k] / (float)sr;
    __syncthreads();
    // (already ascending; the reference's sort_by(partial_cmp) is a no-op here)
    {
        // the HMM grid's frame count (hmm_track's nf) bounds its beats: LDS when it fits
        const float interval = 60.0f / bpm;
        const uint64_t nfr = sd_f2u64(__builtin_ceilf((onp[n - 1] - onp[0]) / interval)) + 1;
        if (bpm > EPS && nfr <= (uint64_t)BEAT_LDS_B) hb = s_hb;
    }
    int nh = hmm_track(bpm, onp, n, hb, cap, &overflow);
    __syncthreads();
    if (nh <= 0 || overflow) {
        if (overflow) r.ok = -1;
        finish();
        return;
    }
    const float* fin = hb;
    int nfin = nh;
    // tempo variations + Bayesian refinement (mod.rs:140-219); every lane replays the segment
    // generator identically (uniform control flow)
    SegGen g;
    if (!seg_init(g, hb, nh, bpm)) {
        finish();
        return;
    }
    bool any = false, has_var = false;
    Seg s;
    {
        SegGen g2 = g;
        bool any2 = false;
        while (seg_next(g2, &s, &any2)) has_var |= s.variable;
    }
    if (has_var) {
        float cur_bpm = bpm;
        int nr = 0;
        while (seg_next(g, &s, &any)) {
            if (s.variable) {
                const int i0 = lower_bound_f(onp, n, s.start);
                const int i1 = upper_bound_f(onp, n, s.end);
                if (i1 > i0) {
                    float ub;
                    if (!bayes_update(&cur_bpm, onp + i0, i1 - i0, &ub)) {
                        finish();  // Err propagates -> empty grid
                        return;
                    }
                    const int got = hmm_track(ub, onp + i0, i1 - i0, rb + nr, cap - nr, &overflow);
                    __syncthreads();
                    if (overflow) {
                        r.ok = -1;
                        finish();
                        return;
                    }
                    if (got > 0) nr += got;
                }
            } else {
                const int j0 = lower_bound_f(hb, nh, s.start);
                const int j1 = upper_bound_f(hb, nh, s.end);
                if (nr + (j1 - j0) > cap) {
                    r.ok = -1;
                    finish();
                    return;
                }
                for (int k = j0 + lane; k < j1; k += 64) rb[nr + (k - j0)] = hb[k];
                nr += j1 - j0;
                __syncthreads();
            }
        }
        if (nr > 0) {
            int np2 = 1;
            while (np2 < nr) np2 <<= 1;
            if (np2 <= BEAT_SORT_MAX) {
                wave_sort_stable(rb, s_rb, nr, s_kv, s_ki, np2);
                fin = s_rb;
            } else {
                if (lane == 0) merge_sort_f(rb, tmp, nr);
                __syncthreads();
                fin = rb;
            }
            nfin = nr;
        }
    }
    // time signature (time_signature.rs:90-149): lanes 0/1/2 score 4/4, 3/4, 6/8
    int bpb = 4;
    if (nfin >= 8) {
        float sum = 0.0f;
        int niv = 0;
        for (int k = 1; k < nfin; k++) {
            const float d = fin[k] - fin[k - 1];
            if (d > 0.0f) {
                sum += d;
                niv++;
            }
        }
        if (niv > 0) {
            const float mean = sum / (float)niv;
            float sc = 0.0f;
            if (lane < 3) sc = score_ts(fin, nfin, lane == 0 ? 4 : lane == 1 ? 3 : 6, mean, niv);
            const float s44 = __shfl(sc, 0, 64), s34 = __shfl(sc, 1, 64), s68 = __shfl(sc, 2, 64);
            float bs = s44;
            if (!(s34 < bs)) {
                bpb = 3;
                bs = s34;
            }
            if (!(s68 < bs)) {
                bpb = 6;
                bs = s68;
            }
        }
    }
    // beats + downbeats (mod.rs:290-404)
    for (int k = lane; k < nfin; k += 64) ob[k] = fin[k];
    int nd = 0;
    if (lane == 0) {
        const float bi = 60.0f / bpm;
        const float bar = bi * (float)bpb;
        const float tolb = bar * 0.1f;
        float last = fin[0];
        od[nd++] = last;
        for (int k = 1; k < nfin; k++) {
            const float et = last + bar;
            if (sd_absf(fin[k] - et) <= tolb) od[nd++] = last = fin[k];
        }
        // stability (mod.rs:425-485)
        float stab = 0.0f;
        if (nfin >= 2) {
            float sum = 0.0f;
            int niv = 0;
            for (int k = 1; k < nfin; k++) {
                const float d = fin[k] - fin[k - 1];
                if (d > 0.0f) {
                    sum += d;
                    niv++;
                }
            }
            if (niv > 0) {
                const float mean = sum / (float)niv;
                if (mean > 1e-10f) {
                    float vs = 0.0f;
                    for (int k = 1; k < nfin; k++) {
                        const float d = fin[k] - fin[k - 1];
                        if (d > 0.0f) {
                            const float dd = d - mean;
                            vs += dd * dd;
                        }
                    }
                    const float var = vs / (float)niv;
                    const float cv = __builtin_sqrtf(var) / mean;
                    stab = 1.0f / (1.0f + cv);
                }
            }
        }
        r.n_beats = nfin;
        r.n_down = nd;
        r.stability = stab;
        r.ok = 1;
        out[trk] = r;
    }
}

void launch_beat(const int* tracks, int n_items, const uint32_t* onsets, const uint64_t* on_off, const int* on_n,
                 uint32_t sr, const float* bpm, const float* conf, float* scratch, const uint64_t* beat_off,
                 const int* beat_cap, float* beats, float* downs, BeatOut* out, hipStream_t st) {
    if (n_items == 0) return;
    hipLaunchKernelGGL(k_beat, dim3(n_items), dim3(64), 0, st, tracks, n_items, onsets, on_off, on_n, sr,
                       bpm, conf, scratch, beat_off, beat_cap, beats, downs, out);
}

// Gathers the tracks' beat and downbeat lists (capacity-strided in `beats` / `downs`) into
// dense arrays so the host downloads only what was produced: one workgroup; pfx[0..n] and
// pfx[n+1..2n+1] are the exclusive prefixes of the beat and downbeat counts (0 for failed
// tracks).  Integer sums, so the scan order is immaterial.
__global__ __launch_bounds__(1024) void k_beat_compact(int n, const BeatOut* __restrict__ out,
                                                       const uint64_t* __restrict__ beat_off,
                                                       const float* __restrict__ beats, const float* __restrict__ downs,
                                                       uint64_t* __restrict__ pfx, float* __restrict__ cb,
                                                       float* __restrict__ cd) {
    __shared__ uint64_t sb[1024], sd[1024];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int per = (n + nt - 1) / nt, i0 = tid * per, i1 = min(n, i0 + per);
    uint64_t ab = 0, ad = 0;
    for (int i = i0; i < i1; i++) {
        const BeatOut r = out[i];
        ab += r.ok > 0 ? (uint64_t)r.n_beats : 0;
        ad += r.ok > 0 ? (uint64_t)r.n_down : 0;
    }
    sb[tid] = ab;
    sd[tid] = ad;
    __syncthreads();
    for (int o = 1; o < nt; o <<= 1) {  // inclusive Hillis-Steele scan
        const uint64_t vb = tid >= o ? sb[tid - o] : 0, vd = tid >= o ? sd[tid - o] : 0;
        __syncthreads();
        sb[tid] += vb;
        sd[tid] += vd;
        __syncthreads();
    }
    uint64_t pb = sb[tid] - ab, pd = sd[tid] - ad;
    for (int i = i0; i < i1; i++) {
        const BeatOut r = out[i];
        pfx[i] = pb;
        pfx[n + 1 + i] = pd;
        pb += r.ok > 0 ? (uint64_t)r.n_beats : 0;
        pd += r.ok > 0 ? (uint64_t)r.n_down : 0;
    }
    if (tid == nt - 1) {
        pfx[n] = sb[tid];
        pfx[2 * n + 1] = sd[tid];
    }
    __syncthreads();
    const int lane = tid & 63, w = tid >> 6, nw = nt >> 6;
    for (int i = w; i < n; i += nw) {  // one wave per track
        const BeatOut r = out[i];
        if (r.ok <= 0) continue;
        const uint64_t ob = pfx[i], od = pfx[n + 1 + i], src = beat_off[i];
        for (int k = lane; k < r.n_beats; k += 64) cb[ob + k] = beats[src + k];
        for (int k = lane; k < r.n_down; k += 64) cd[od + k] = downs[src + k];
    }
}

// The same gather with one 64-thread workgroup per track: the wave sums the counts of the tracks
// before its own (n/64 loads per lane, L2-resident) and copies its track.  A single-wave
// workgroup dispatches into any free wave slot, where the 1024-thread one above waits for 16 slots
// on one CU; on the shared chip (the key stream's STFT holds most slots) that wait stalled the
// tempo stream behind it.  Used up to COMPACT_W_MAX tracks (the prefix work is quadratic in n).
constexpr int COMPACT_W_MAX = 4096;
__global__ __launch_bounds__(64) void k_beat_compact_w(int n, const BeatOut* __restrict__ out,
                                                       const uint64_t* __restrict__ beat_off,
                                                       const float* __restrict__ beats, const float* __restrict__ downs,
                                                       uint64_t* __restrict__ pfx, float* __restrict__ cb,
                                                       float* __restrict__ cd) {
    const int i = blockIdx.x, lane = threadIdx.x;
    uint64_t ab = 0, ad = 0;
    for (int j = lane; j < i; j += 64) {
        const BeatOut r = out[j];
        ab += r.ok > 0 ? (uint64_t)r.n_beats : 0;
        ad += r.ok > 0 ? (uint64_t)r.n_down : 0;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        ab += __shfl_xor(ab, o, 64);
        ad += __shfl_xor(ad, o, 64);
    }
    const BeatOut r = out[i];
    const uint64_t nb = r.ok > 0 ? (uint64_t)r.n_beats : 0, nd = r.ok > 0 ? (uint64_t)r.n_down : 0;
    if (lane == 0) {
        pfx[i] = ab;
        pfx[n + 1 + i] = ad;
        if (i == n - 1) {
            pfx[n] = ab + nb;
            pfx[2 * n + 1] = ad + nd;
        }
    }
    if (r.ok <= 0) return;
    const uint64_t src = beat_off[i];
    for (int k = lane; k < r.n_beats; k += 64) cb[ab + k] = beats[src + k];
    for (int k = lane; k < r.n_down; k += 64) cd[ad + k] = downs[src + k];
}

void launch_beat_compact(int n, const BeatOut* out, const uint64_t* beat_off, const float* beats, const float* downs,
                         uint64_t* pfx, float* cb, float* cd, hipStream_t st) {
    if (n == 0) return;
    if (n <= COMPACT_W_MAX)
        hipLaunchKernelGGL(k_beat_compact_w, dim3(n), dim3(64), 0, st, n, out, beat_off, beats, downs, pfx, cb, cd);
    else
        hipLaunchKernelGGL(k_beat_compact, dim3(1), dim3(1024), 0, st, n, out, beat_off, beats, downs, pfx, cb, cd);
}

}  // namespace sdsp
