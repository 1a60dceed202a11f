// k_frontend.hip — preprocessing and onset front-end kernels.
//
//   k_peak_abs / k_gain      normalize_peak            src/preprocessing/normalization.rs:262-322
//   k_loudness_gain          normalize_rms / _lufs     normalization.rs:119-259, 325-470
//   k_frame_rms              frame RMS                 silence.rs:154-169, energy_flux.rs:122-131
//   k_trim                   silence regions + trim    silence.rs:171-279
//   k_energy_onsets          energy-flux onsets        energy_flux.rs:133-243
//   k_flux_onsets            spectral-flux / HFC peaks spectral_flux.rs:160-221, hfc.rs:156-214
//   k_consensus              onset voting + selection  consensus.rs:111-287, src/lib.rs:181-290
//
// The normalised signal is never materialised: every consumer reads raw*gain (one f32
// multiply, exactly the value the reference stores in place).
#include "block_utils.hpp"
#include <cstdlib>

#include "kernels.hpp"

namespace sdsp {

// ---- peak |x| per track (an order-free max of |x| >= 0, taken on the IEEE bits) ----
// PK_CH samples per workgroup: the 16-B aligned body as float4 loads, all PK_U of a thread in
// flight at once (a 4-B stream kept too few bytes in flight to reach HBM bandwidth); the < 4
// unaligned samples at either end as scalars.  Each workgroup writes its chunk's maximum and
// k_peak_fold takes the maximum over a track's chunks: the round-3 form, one atomicMax per wave
// on the track's word, serialised the ~2,000 waves of a track on one L2 line (k_peak_abs lasted
// ~25 us per workgroup whatever its size).
constexpr int PK_U = PK_CH / (4 * 256);  // float4 loads per thread
static_assert(PK_U * 4 * 256 == PK_CH, "PK_CH = 1024 * PK_U");
__global__ __launch_bounds__(256) void k_peak_abs(const float* __restrict__ x, const uint64_t* __restrict__ in_off,
                                                  const uint64_t* __restrict__ n_raw,
                                                  const uint64_t* __restrict__ chunk_pfx, int T,
                                                  unsigned int* __restrict__ chunk_bits) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ float wmax[4];
    const uint64_t g = blockIdx.x;
    const int trk = find_track(chunk_pfx, T, g);
    const uint64_t c = g - chunk_pfx[trk];
    const uint64_t s0 = c * PK_CH, n = n_raw[trk];
    const int64_t len = (int64_t)((s0 + PK_CH < n ? s0 + PK_CH : n) - s0);
    const float* p = x + in_off[trk] + s0;
    const int lead = (int)(((16u - ((uintptr_t)p & 15u)) & 15u) / 4u);  // samples before 16-B alignment
    const int64_t h = lead < len ? lead : len;
    const int64_t nb = (len - h) / 4;  // aligned float4s
    // with no aligned float4 the clamped loads below read the 16-B block holding p[0], which lies
    // inside the allocation like p[0] itself
    const f4* q = reinterpret_cast<const f4*>(nb > 0 ? p + h : (const float*)((uintptr_t)p & ~(uintptr_t)15));
    const int tid = threadIdx.x;
    float m = 0.0f;
    f4 v[PK_U];
#pragma unroll
    for (int u = 0; u < PK_U; u++) {
        const int64_t k = tid + 256 * u;  // clamped unconditional load, then a select (no per-load wait)
        const f4 qv = q[k < nb ? k : (nb > 0 ? nb - 1 : 0)];  // nb == 0: q[0], see above
        v[u] = k < nb ? qv : f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    if (tid < h) m = sd_absf(p[tid]);
    const int64_t tl = h + 4 * nb;
    if (tid < len - tl) m = sd_maxf(m, sd_absf(p[tl + tid]));
#pragma unroll
    for (int u = 0; u < PK_U; u++)
        m = sd_maxf(m, sd_maxf(sd_maxf(sd_absf(v[u].x), sd_absf(v[u].y)), sd_maxf(sd_absf(v[u].z), sd_absf(v[u].w))));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) chunk_bits[g] = sd_bits_f(sd_maxf(sd_maxf(wmax[0], wmax[1]), sd_maxf(wmax[2], wmax[3])));
}

// peak_bits[t] = the maximum of track t's chunk maxima (every one a float >= +0 or +inf, so the
// unsigned maximum of the bits is the float maximum), one wave per track
__global__ __launch_bounds__(64) void k_peak_fold(const uint64_t* __restrict__ chunk_pfx, int T,
                                                  const unsigned int* __restrict__ chunk_bits,
                                                  unsigned int* __restrict__ peak_bits) {
    const int t = blockIdx.x;
    if (t >= T) return;
    unsigned int m = 0;
    for (uint64_t c = chunk_pfx[t] + threadIdx.x; c < chunk_pfx[t + 1]; c += 64) m = max(m, chunk_bits[c]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
    if (threadIdx.x == 0) peak_bits[t] = m;
}

// gain = min(10^(-headroom/20)/peak, 1/peak); peak <= 1e-10 leaves the samples untouched.
__global__ void k_gain(const unsigned int* __restrict__ peak_bits, int T, float target, int enable,
                       float* __restrict__ gain) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const float peak = sd_from_bits_f(peak_bits[t]);
    float g = 1.0f;
    if (enable && peak > EPS) g = sd_minf(target / peak, 1.0f / peak);
    gain[t] = g;
}

// Silence regions and trim bounds (silence.rs:171-279), one workgroup per track.  Only two
// regions can move the trim: the run of silent frames starting at frame 0 (always kept, its
// end becomes the trim start) and the run reaching the last frame (kept when at least
// min_frames long or starting at 0; its start becomes the trim end).  Both follow from the
// first and the last non-silent frame, found by an order-free min/max reduction.
__global__ __launch_bounds__(256) void k_trim(const float* __restrict__ rms, const uint64_t* __restrict__ frame_pfx,
                                              const uint64_t* __restrict__ base_pfx, int stride,
                                              int T, const uint64_t* __restrict__ n_raw, int hop, float thr,
                                              uint64_t min_frames, int enable, uint64_t* __restrict__ trim_start,
                                              uint64_t* __restrict__ trim_end) {
    SDSP_LATENCY_CRITICAL();
    __shared__ long long red_lo[4], red_hi[4];
    const int t = blockIdx.x;
    const uint64_t n = n_raw[t];
    if (!enable || n == 0) {
        if (threadIdx.x == 0) {
            trim_start[t] = 0;
            trim_end[t] = n;
        }
        return;
    }
    const int64_t nf = (int64_t)(frame_pfx[t + 1] - frame_pfx[t]);
    const float* r = rms + base_pfx[t];  // frame f at r[f * stride]
    long long lo = nf, hi = -1;  // first / last non-silent frame
    for (int64_t f = threadIdx.x; f < nf; f += blockDim.x)
        if (!(r[f * stride] <= thr)) {
            lo = lo < f ? lo : f;
            hi = hi > f ? hi : f;
        }
    for (int o = 32; o > 0; o >>= 1) {
        const long long l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
        lo = lo < l2 ? lo : l2;
        hi = hi > h2 ? hi : h2;
    }
    if ((threadIdx.x & 63) == 0) {
        red_lo[threadIdx.x >> 6] = lo;
        red_hi[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
        lo = red_lo[0] < red_lo[w] ? red_lo[0] : red_lo[w];
        red_lo[0] = lo;
        hi = red_hi[0] > red_hi[w] ? red_hi[0] : red_hi[w];
        red_hi[0] = hi;
    }
    lo = red_lo[0];
    hi = red_hi[0];
    uint64_t ts = 0, te = n;
    if (nf > 0 && lo > 0) ts = lo < nf ? (uint64_t)lo * (uint64_t)hop : n;  // frame 0 silent
    if (nf > 0 && hi < nf - 1) {                                             // last frame silent
        const uint64_t ss = (uint64_t)(hi + 1);
        if ((uint64_t)nf - ss >= min_frames || ss == 0) te = ss * (uint64_t)hop;
    }
    if (ts > te) ts = te;
    if (te < ts) te = ts;
    if (!(ts < te && te <= n)) ts = te = 0;
    trim_start[t] = ts;
    trim_end[t] = te;
}

// Energy-flux onsets (energy_flux.rs:133-243).  rms: per-frame RMS (frame_size, hop) of the
// trimmed signal.  Out: onset sample positions (relative to the trimmed start), ascending.
__global__ __launch_bounds__(256) void k_energy_onsets(const float* __restrict__ rms,
                                                       const uint64_t* __restrict__ frame_pfx,
                                                       const uint64_t* __restrict__ n_trim, int hop, float factor,
                                                       uint32_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                       int* __restrict__ out_n) {
    SDSP_LATENCY_CRITICAL();
    __shared__ float redf[8];
    __shared__ int redi[9];
    const int trk = blockIdx.x;
    const int64_t nf = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const float* e = rms + frame_pfx[trk];
    const uint64_t n = n_trim[trk];
    uint32_t* o = out + out_off[trk];
    if (nf < 2) {
        if (threadIdx.x == 0) out_n[trk] = 0;
        return;
    }
    const int64_t L = nf - 1;
    auto flux = [&](int64_t i) { return sd_maxf(e[i + 1] - e[i], 0.0f); };
    float m = 0.0f;
    for (int64_t i = threadIdx.x; i < L; i += blockDim.x) m = sd_maxf(m, flux(i));
    m = block_max(m, redf);
    if (m <= EPS) {
        if (threadIdx.x == 0) out_n[trk] = 0;
        return;
    }
    const float thr = m * factor;
    int base = 0;
    for (int64_t c0 = 0; c0 < L; c0 += blockDim.x) {
        const int64_t i = c0 + threadIdx.x;
        bool on = false;
        if (i < L && L > 1) {
            const float f = flux(i);
            if (i == 0)
                on = f > thr && f >= flux(1);
            else if (i == L - 1)
                on = f > thr && f > flux(i - 1);
            else
                on = f > thr && f > flux(i - 1) && f >= flux(i + 1);
            on = on && (uint64_t)(i + 1) * (uint64_t)hop < n;
        }
        int total;
        const int slot = block_exclusive_flag(on, redi, &total);
        if (on) o[base + slot] = (uint32_t)((i + 1) * hop);
        base += total;
    }
    if (threadIdx.x == 0) out_n[trk] = base;
}

// Spectral-flux (kind 0), HFC (kind 1) or HPSS (kind 2) onsets: percentile threshold + local
// peaks, as sample positions f*hop < n (spectral_flux.rs:160-215, hfc.rs:156-208,
// hpss.rs:318-368, src/lib.rs:181-236).  sfo: per-frame-pair spectral flux (index t-1 for pair
// (t-1,t)); hfc: per-frame HFC; hpe: per-frame energy of the percussive spectrogram.
__global__ __launch_bounds__(256) void k_flux_onsets(const float* __restrict__ sfo, const float* __restrict__ hfc,
                                                     const float* __restrict__ hpe, float* __restrict__ scratch,
                                                     const uint64_t* __restrict__ frame_pfx,
                                                     const uint64_t* __restrict__ n_trim, int hop, float pct,
                                                     uint32_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                     int* __restrict__ out_n, int T) {
    SDSP_LATENCY_CRITICAL();
    __shared__ int hist[256];
    __shared__ int misc[4];
    __shared__ int redi[9];
    const int trk = blockIdx.x % T;
    const int kind = blockIdx.x / T;
    const int64_t nf = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    uint32_t* o = out + out_off[trk] + (uint64_t)kind * (frame_pfx[T]);  // kind-major halves
    int* on_n = out_n + kind * T;
    if (nf < 2) {
        if (threadIdx.x == 0) on_n[trk] = 0;
        return;
    }
    const int64_t L = nf - 1;
    float* fl = scratch + frame_pfx[trk] + (uint64_t)kind * frame_pfx[T];
    if (kind == 0) {
        const float* s = sfo + frame_pfx[trk];
        for (int64_t i = threadIdx.x; i < L; i += blockDim.x) fl[i] = s[i];
    } else {  // kind 1: HFC flux (hfc.rs:143-146); kind 2: percussive energy flux (hpss.rs:311-316)
        const float* h = (kind == 1 ? hfc : hpe) + frame_pfx[trk];
        for (int64_t i = threadIdx.x; i < L; i += blockDim.x) fl[i] = sd_maxf(h[i + 1] - h[i], 0.0f);
    }
    __syncthreads();
    uint64_t ti = sd_f2u64((float)L * pct);
    if (ti > (uint64_t)(L - 1)) ti = (uint64_t)(L - 1);
    const float thr = block_select_kth(fl, (int)L, (int)ti, hist, misc);
    const uint64_t n = n_trim[trk];
    int base = 0;
    for (int64_t c0 = 0; c0 < L; c0 += blockDim.x) {
        const int64_t i = c0 + threadIdx.x;
        bool on = false;
        if (i < L && L > 1) {
            const float f = fl[i];
            if (i == 0)
                on = f > thr && f >= fl[1];
            else if (i == L - 1)
                on = f > thr && f > fl[i - 1];
            else
                on = f > thr && f > fl[i - 1] && f >= fl[i + 1];
            on = on && (uint64_t)(i + 1) * (uint64_t)hop < n;  // frame i+1 -> sample (i+1)*hop
        }
        int total;
        const int slot = block_exclusive_flag(on, redi, &total);
        if (on) o[base + slot] = (uint32_t)((i + 1) * hop);
        base += total;
    }
    if (threadIdx.x == 0) on_n[trk] = base;
}

// Onset consensus (consensus.rs:111-287) + selection (src/lib.rs:258-290), one workgroup per
// track.  The reference merges the three sorted lists (stable: energy, spectral, HFC on equal
// samples) and joins each onset to the first cluster with a member within tol.  Onsets arrive
// sorted, so a new cluster is only ever created once every earlier cluster is out of reach:
// joining reduces to comparing against the newest cluster's largest member, i.e. a new
// cluster starts wherever the gap to the previous merged onset exceeds tol.  Every cluster is
// a maximal run of the merged order (and the integer centres strictly increase), so it
// parallelises exactly: merged positions by rank (binary searches), cluster starts by
// ordered compaction, integer sums per cluster, then the strong (>= 2 methods) centres, or
// all centres when none is strong, or the energy onsets when nothing clustered.
// scr: 5 * (3F) uint32 per track at scr_off (merged value, method, cluster start, centre, strong).
__device__ inline int lb_u32(const uint32_t* a, int n, uint32_t x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ inline int ub_u32(const uint32_t* a, int n, uint32_t x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (!(x < a[mid])) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_consensus(const uint32_t* __restrict__ energy,
                                                   const uint64_t* __restrict__ e_off, const int* __restrict__ e_n,
                                                   const uint32_t* __restrict__ flux_on,
                                                   const uint64_t* __restrict__ f_off, const int* __restrict__ f_n,
                                                   uint64_t kind_stride, int T, uint32_t tol, int enable,
                                                   const int* __restrict__ has_mags, uint32_t* __restrict__ chosen,
                                                   const uint64_t* __restrict__ c_off, int* __restrict__ c_n,
                                                   uint32_t* __restrict__ scr, int hpss) {
    SDSP_LATENCY_CRITICAL();
    __shared__ int red[8];
    const int t = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t* L0 = energy + e_off[t];
    const int n0 = e_n[t];
    uint32_t* out = chosen + c_off[t];
    auto keep_energy = [&]() {
        for (int i = tid; i < n0; i += blockDim.x) out[i] = L0[i];
        if (tid == 0) c_n[t] = n0;
    };
    if (!enable || !has_mags[t]) {
        keep_energy();
        return;
    }
    const uint32_t* L1 = flux_on + f_off[t];
    const uint32_t* L2 = flux_on + f_off[t] + kind_stride;
    const uint32_t* L3 = flux_on + f_off[t] + 2 * kind_stride;  // HPSS onsets (kind 2) when enabled
    const int n1 = f_n[t], n2 = f_n[T + t], n3 = hpss ? f_n[2 * T + t] : 0;
    const int N = n0 + n1 + n2 + n3;
    const uint64_t cap = (uint64_t)N > 0 ? (uint64_t)N : 1;
    uint32_t* mv = scr + c_off[t] * 5;  // c_off = (3 or 4) * frame offset: 3F / 4F slots per array
    uint32_t* mm = mv + cap;
    uint32_t* cs = mm + cap;
    uint32_t* cc = cs + cap;
    uint32_t* sg = cc + cap;
    // merged order by rank
    for (int e = tid; e < N; e += blockDim.x) {
        int a, i;
        uint32_t s;
        if (e < n0) {
            a = 0;
            i = e;
            s = L0[i];
        } else if (e < n0 + n1) {
            a = 1;
            i = e - n0;
            s = L1[i];
        } else if (e < n0 + n1 + n2) {
            a = 2;
            i = e - n0 - n1;
            s = L2[i];
        } else {
            a = 3;
            i = e - n0 - n1 - n2;
            s = L3[i];
        }
        int pos = i;  // stable merge rank: earlier lists win ties
        pos += a == 0 ? 0 : ub_u32(L0, n0, s);
        pos += a == 1 ? 0 : (a < 1 ? lb_u32(L1, n1, s) : ub_u32(L1, n1, s));
        pos += a == 2 ? 0 : (a < 2 ? lb_u32(L2, n2, s) : ub_u32(L2, n2, s));
        pos += a == 3 ? 0 : lb_u32(L3, n3, s);
        mv[pos] = s;
        mm[pos] = (uint32_t)a;
    }
    __syncthreads();
    // cluster starts, in order
    int C = 0;
    for (int p0 = 0; p0 < N; p0 += blockDim.x) {
        const int p = p0 + tid;
        const bool st = p < N && (p == 0 || (uint64_t)(mv[p] - mv[p - 1]) > (uint64_t)tol);
        int tot;
        const int slot = block_exclusive_flag(st, red, &tot);
        if (st) cs[C + slot] = (uint32_t)p;
        C += tot;
    }
    __syncthreads();
    // per-cluster centre and vote
    for (int c = tid; c < C; c += blockDim.x) {
        const int b = (int)cs[c], e = c + 1 < C ? (int)cs[c + 1] : N;
        uint64_t sum = 0;
        int voted = 0;
        for (int p = b; p < e; p++) {
            sum += mv[p];
            voted |= 1 << mm[p];
        }
        cc[c] = (uint32_t)(sum / (uint64_t)(e - b));
        sg[c] = __popc(voted) >= 2;
    }
    __syncthreads();
    // pass 1: strong centres, consecutive duplicates dropped
    int K = 0;
    for (int c0 = 0; c0 < C; c0 += blockDim.x) {
        const int c = c0 + tid;
        const bool f = c < C && sg[c];
        int tot;
        const int slot = block_exclusive_flag(f, red, &tot);
        if (f) mv[K + slot] = cc[c];  // mv is free now
        K += tot;
    }
    __syncthreads();
    const uint32_t* src = mv;
    int S = K;
    if (K == 0) {  // no strong cluster: every centre
        src = cc;
        S = C;
    }
    int ns = 0;
    for (int k0 = 0; k0 < S; k0 += blockDim.x) {
        const int k = k0 + tid;
        const bool f = k < S && (k == 0 || src[k] != src[k - 1]);
        int tot;
        const int slot = block_exclusive_flag(f, red, &tot);
        if (f) out[ns + slot] = src[k];
        ns += tot;
    }
    if (ns == 0) {  // nothing clustered: keep the energy-flux onsets (lib.rs:283-285)
        keep_energy();
        return;
    }
    if (tid == 0) c_n[t] = ns;
}

// ---- launchers ----
static void launch_peak(const float* x, const uint64_t* in_off, const uint64_t* n_raw, const uint64_t* chunk_pfx, int T,
                        uint64_t n_chunks, unsigned int* chunk_bits, unsigned int* peak_bits, hipStream_t st) {
    if (n_chunks) hipLaunchKernelGGL(k_peak_abs, dim3((unsigned)n_chunks), dim3(256), 0, st, x, in_off, n_raw, chunk_pfx, T, chunk_bits);
    hipLaunchKernelGGL(k_peak_fold, dim3((unsigned)T), dim3(64), 0, st, chunk_pfx, T, chunk_bits, peak_bits);
}
void launch_peak_gain(const float* x, const uint64_t* in_off, const uint64_t* n_raw, const uint64_t* chunk_pfx, int T,
                      uint64_t n_chunks, unsigned int* chunk_bits, unsigned int* peak_bits, float target, int enable,
                      float* gain, hipStream_t st) {
    if (T == 0) return;
    launch_peak(x, in_off, n_raw, chunk_pfx, T, n_chunks, chunk_bits, peak_bits, st);
    hipLaunchKernelGGL(k_gain, dim3((T + 255) / 256), dim3(256), 0, st, peak_bits, T, target, enable, gain);
}
// ---- RMS / LUFS gain (normalization.rs:325-470): one lane per track ----
// Both methods fold the whole track in sample order (the f32 sum of squares, and the K-weighting
// biquad, a recurrence), so the fold itself is one lane per track.  A workgroup owns LG_TPW
// tracks: lanes 0..LG_TPW-1 of wave 0 fold them while LG_LOADERS loader waves stage the next
// LG_C-sample chunk of every track into the other half of a double-buffered LDS tile.  Each load
// instruction reads 1 KB (aligned track) or 256 B (unaligned) of ONE track: a lane-per-track
// global stream touches a page per lane per instruction and is TLB-bound, and the fold wave
// alone cannot keep enough bytes in flight.  The LUFS lane runs the biquad, folds each 400-ms
// block's mean square at its end and gates it on the fly, so nothing but the gain leaves the
// lane.  The peak comes from k_peak_abs.
constexpr int LG_TPW = 16;          // tracks per workgroup
constexpr int LG_C = 1024;          // samples per track per chunk
constexpr int LG_ROW = LG_C + 4;    // LDS row stride (floats): rows start 4 banks apart
constexpr int LG_LOADERS = 8;       // loader waves
template <bool RMS>
__global__ __launch_bounds__(64 * (1 + LG_LOADERS)) void k_loudness_gain(
    const float* __restrict__ x, const uint64_t* __restrict__ in_off, const uint64_t* __restrict__ n_raw, int T,
    const unsigned int* __restrict__ peak_bits, LoudnessParams P, float* __restrict__ gain, int* __restrict__ status) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    extern __shared__ float lg_tile[];  // [2][LG_TPW][LG_ROW]
    __shared__ uint64_t nmax_s, nmin_s;
    const int w = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int t0 = blockIdx.x * LG_TPW;
    const int nt = T - t0 < LG_TPW ? T - t0 : LG_TPW;
    if (threadIdx.x == 0) nmax_s = 0, nmin_s = ~0ull;
    __syncthreads();
    if (w == 0 && lane < nt) {
        atomicMax((unsigned long long*)&nmax_s, (unsigned long long)n_raw[t0 + lane]);
        atomicMin((unsigned long long*)&nmin_s, (unsigned long long)n_raw[t0 + lane]);
    }
    __syncthreads();
    const uint64_t nch = (nmax_s + LG_C - 1) / LG_C;
    auto load = [&](uint64_t c, int buf) {  // loader waves: chunk c of every track
        float* base = lg_tile + (size_t)buf * LG_TPW * LG_ROW;
        const uint64_t s0 = c * LG_C;
        for (int tt = w - 1; tt < nt; tt += LG_LOADERS) {
            const uint64_t a = in_off[t0 + tt], n = n_raw[t0 + tt];
            float* row = base + tt * LG_ROW;
            if ((a & 3u) == 0 && s0 + LG_C <= n) {  // whole aligned chunk: 16-B loads
                const f4* q = reinterpret_cast<const f4*>(x + a + s0);
                f4 v[LG_C / 256];
#pragma unroll
                for (int i = 0; i < LG_C / 256; i++) v[i] = q[i * 64 + lane];
#pragma unroll
                for (int i = 0; i < LG_C / 256; i++) reinterpret_cast<f4*>(row)[i * 64 + lane] = v[i];
            } else {
                float v[LG_C / 64];
#pragma unroll
                for (int i = 0; i < LG_C / 64; i++) {
                    const uint64_t sm = s0 + (uint64_t)(i * 64 + lane);
                    v[i] = sm < n ? x[a + sm] : 0.0f;
                }
#pragma unroll
                for (int i = 0; i < LG_C / 64; i++) row[i * 64 + lane] = v[i];
            }
        }
    };
    if (w > 0 && nch > 0) load(0, 0);
    __syncthreads();

    // ---- wave 0: the per-track folds ----
    // Every track starts at sample 0 and chunk c covers samples [c*LG_C, (c+1)*LG_C) of every
    // track, so the position inside the 400-ms block is the same for all lanes: the block
    // bookkeeping is wave-uniform (scalar branches, no exec-mask divergence), and a chunk that
    // every track fills completely runs without per-lane tests.
    const bool act = w == 0 && lane < nt;
    const uint64_t n = act ? n_raw[t0 + lane] : 0;
    const float b0 = P.b0, b1 = P.b1, b2 = P.b2, a1 = P.a1, a2 = P.a2;
    const int64_t bs = P.block;
    constexpr bool rms = RMS;
    float ss = 0.0f;                                        // RMS: sum of squares
    // LUFS: biquad state (x1, x2), block and gated sums.  The state update is written on f32
    // pairs so that it issues as packed ops (v_pk_add/mul_f32, each lane of a pair rounded
    // exactly like the scalar op): (o, t) = (x1, x2) + (b0 v, b1 v); (x1, x2) = (t, b2 v) -
    // (a1 o, a2 o) -- the reference's `b0*s + x1`, `b1*s + x2 - a1*o`, `b2*s - a2*o`.
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 xs = {0.0f, 0.0f};
    const f2 B01 = {b0, b1}, A12 = {a1, a2};
    float bsum = 0.0f, gsum = 0.0f;
    int64_t cnt = 0;  // samples into the current block (uniform)
    int gn = 0;
    auto biquad = [&](float v) {  // Direct Form II transposed, KWeightingFilter::process
        const f2 vv = {v, v};
        const f2 ot = B01 * vv + xs;
        const f2 oo = {ot.x, ot.x};
        const f2 tb = {ot.y, b2 * v};
        xs = tb - A12 * oo;
        bsum += ot.x * ot.x;
    };
    auto step = [&](float v) {
        if (rms)
            ss += v * v;
        else
            biquad(v);
    };
    auto close_block = [&](int64_t len) {
        const float ms = bsum / (float)len;
        if (ms > P.gate) {
            gsum += ms;
            gn++;
        }
        bsum = 0.0f;
    };
    for (uint64_t c = 0; c < nch; c++) {
        const int buf = (int)(c & 1);
        if (w > 0) {
            if (c + 1 < nch) load(c + 1, buf ^ 1);
        } else {
            const float* row = lg_tile + (size_t)buf * LG_TPW * LG_ROW + lane * LG_ROW;
            const f4* row4 = reinterpret_cast<const f4*>(row);
            const uint64_t s0 = c * LG_C;
            if (s0 + LG_C <= nmin_s) {  // every track fills this chunk
                int i = 0;
                while (i < LG_C) {
                    // samples up to the next block end (or the chunk end), uniform
                    const int64_t room = rms ? (int64_t)LG_C : bs - cnt;
                    const int e = (int64_t)(LG_C - i) < room ? LG_C : i + (int)room;
                    int k = i;
                    for (; k < e && (k & 3); k++) step(row[k]);
                    for (; k + 16 <= e; k += 16) {
                        const f4 v0 = row4[k / 4], v1 = row4[k / 4 + 1], v2 = row4[k / 4 + 2], v3 = row4[k / 4 + 3];
                        step(v0.x), step(v0.y), step(v0.z), step(v0.w);
                        step(v1.x), step(v1.y), step(v1.z), step(v1.w);
                        step(v2.x), step(v2.y), step(v2.z), step(v2.w);
                        step(v3.x), step(v3.y), step(v3.z), step(v3.w);
                    }
                    for (; k + 4 <= e; k += 4) {
                        const f4 v = row4[k / 4];
                        step(v.x), step(v.y), step(v.z), step(v.w);
                    }
                    for (; k < e; k++) step(row[k]);
                    if (!rms) {
                        cnt += e - i;
                        if (cnt == bs) {
                            close_block(bs);
                            cnt = 0;
                        }
                    }
                    i = e;
                }
            } else {  // some track ends inside this chunk: per-lane bounds
                const int m = !act || s0 >= n ? 0 : (n - s0 < (uint64_t)LG_C ? (int)(n - s0) : LG_C);
                for (int k = 0; k < LG_C; k++) {
                    if (k < m) step(row[k]);
                    if (!rms && ++cnt == bs) {
                        if (k < m) close_block(bs);
                        cnt = 0;
                    }
                }
            }
        }
        __syncthreads();
    }
    if (!act) return;
    const int t = t0 + lane;
    const float peak = sd_from_bits_f(peak_bits[t]);
    float g = 1.0f;
    int stt = 0;
    if (rms) {  // normalize_rms :325-402
        const float rms = __builtin_sqrtf(ss / (float)n);
        if (rms > EPS) {
            g = P.target_rms / rms;
            if (peak * g > 1.0f) g = 1.0f / peak;
        }
    } else {  // normalize_lufs :405-470 with calculate_lufs :183-259
        const int64_t rem = (int64_t)(n % (uint64_t)bs);
        if (rem > 0) close_block(rem);  // this track's last, partial block
        if (gn == 0) {  // every block under the gate: measured_lufs = -inf -> normalize_peak
            if (peak > EPS) g = sd_minf(P.target_peak / peak, 1.0f / peak);
        } else {
            const float mean = gsum / (float)gn;
            if (mean <= EPS) {
                stt = 1;  // NumericalError("Mean square too small for LUFS calculation")
            } else {
                const float lufs = -0.691f + 10.0f * sd_log10f(mean);
                const float gl = sd_powf(10.0f, (P.target_lufs - lufs) / 20.0f);
                g = peak * gl > P.target_peak ? P.target_peak / peak : gl;
            }
        }
    }
    gain[t] = g;
    status[t] = stt;
}

void launch_loudness_gain(const float* x, const uint64_t* in_off, const uint64_t* n_raw, const uint64_t* chunk_pfx,
                          int T, uint64_t n_chunks, unsigned int* chunk_bits, unsigned int* peak_bits,
                          const LoudnessParams& P, float* gain, int* status, hipStream_t st) {
    if (T == 0) return;
    launch_peak(x, in_off, n_raw, chunk_pfx, T, n_chunks, chunk_bits, peak_bits, st);
    const size_t lds = 2 * LG_TPW * LG_ROW * sizeof(float);
    auto kern = P.method == 1 ? k_loudness_gain<true> : k_loudness_gain<false>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3((T + LG_TPW - 1) / LG_TPW), dim3(64 * (1 + LG_LOADERS)), lds, st, x, in_off, n_raw, T,
                       peak_bits, P, gain, status);
}
// ---- frame RMS: sqrt(sum_{k in frame} (x_k*gain)^2 / len), the sum folded in sample order ----
// Each thread streams its own frame from global memory in 16-B aligned blocks (lanes read
// rows `hop` apart, so every wave-instruction touches 64 lines; 16-B rather than 4-B loads cut
// the instruction count 4x).  hop is a multiple of 4, so a frame's misalignment d is its
// track's; the first block skips its d leading floats and a scalar tail finishes the frame.
constexpr int RMS_U = 8;  // 16-B blocks per step (two steps in flight per thread)
__global__ __launch_bounds__(256) void k_frame_rms(const float* __restrict__ x,
                                                          const uint64_t* __restrict__ src_off,
                                                          const float* __restrict__ gain,
                                                          const uint64_t* __restrict__ n_len,
                                                          const uint64_t* __restrict__ frame_pfx, int T,
                                                          uint64_t total, int fs, int hop, float* __restrict__ rms,
                                                          int only_partial) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const int trk = find_track(frame_pfx, T, g);
    const uint64_t f = g - frame_pfx[trk];
    const uint64_t n = n_len[trk];
    const uint64_t s = f * (uint64_t)hop;
    const uint64_t e = s + (uint64_t)fs < n ? s + (uint64_t)fs : n;
    const int64_t len = e > s ? (int64_t)(e - s) : 0;
    if (only_partial && len == fs) return;  // k_rms_gather took this frame from the raw pass
    const uint64_t a = src_off[trk] + s;  // float index of the frame's first sample
    const int d = (int)(a & 3u);
    const f4* q = reinterpret_cast<const f4*>(x + (a - (uint64_t)d));
    const float gn = gain[trk];
    float sum = 0.0f;
    auto acc = [&](float v) {
        const float y = v * gn;
        sum += y * y;
    };
    // block j holds samples k = 4j - d .. 4j - d + 3
    int64_t j = 0;
    if (d != 0 && len > 0) {
        const f4 h = q[0];
        for (int i = d; i < 4 && i - d < len; i++) acc(h[i]);
        j = 1;
    }
    // RMS_U whole blocks per step, the next step's blocks in flight while this one is folded
    if (4 * (j + RMS_U) - d <= len) {
        f4 cur[RMS_U], nxt[RMS_U];
#pragma unroll
        for (int u = 0; u < RMS_U; u++) cur[u] = q[j + u];
        for (;;) {
            const bool more = 4 * (j + 2 * RMS_U) - d <= len;
            if (more) {
#pragma unroll
                for (int u = 0; u < RMS_U; u++) nxt[u] = q[j + RMS_U + u];
            }
#pragma unroll
            for (int u = 0; u < RMS_U; u++) {
                acc(cur[u].x);
                acc(cur[u].y);
                acc(cur[u].z);
                acc(cur[u].w);
            }
            j += RMS_U;
            if (!more) break;
            for (int u = 0; u < RMS_U; u++) cur[u] = nxt[u];
        }
    }
    for (int64_t k = j == 0 ? 0 : 4 * j - d; k < len; k++) acc(x[a + (uint64_t)k]);  // j == 0: d == 0 or empty
    rms[g] = len > 0 ? __builtin_sqrtf(sum / (float)len) : 0.0f;
}

// Frame RMS as a stream (the default when fs = G * hop, G in {1, 2, 4, 8}, hop a multiple of 32):
// one lane owns RUN = 4 G consecutive frames of a track and reads their samples once, in order
// (RUN 4 G: the shortest run whose (G - 1) / RUN re-read stays small; 8 and 16 measured best for
// the trim (G = 2) and energy (G = 4) passes against 8 / 16 / 32);
// G frames are in progress at any sample, each in its own accumulator, and every sample's
// square is added to all G of them.  Frame j is reset when its first hop-segment starts and
// stored after its G-th, so each accumulator is the frame's own sequential fold in sample order
// (bit-identical to k_frame_rms, which re-reads every sample G times from L2; its overlap
// re-reads mostly miss L2, 33 % hits).  Samples past the track's end load as 0 and add +0.
template <int G>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_frame_rms_run(const float* __restrict__ x, const uint64_t* __restrict__ src_off,
                                                       const float* __restrict__ gain, const uint64_t* __restrict__ n_len,
                                                       const uint64_t* __restrict__ frame_pfx, int T, uint64_t total,
                                                       int fs, int hop, float* __restrict__ rms) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int RUN = 4 * G;
    // the wave-cooperative path's staging tile: per wave, 64 lane rows of 8 16-byte blocks, rows
    // 144 B apart (ds_read_b128 of one block column by 16 lanes then covers all 64 banks)
    __shared__ f4 tile[4][64][9];
    const uint64_t u0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * RUN;
    const uint64_t u1 = u0 + RUN < total ? u0 + RUN : total;
    uint64_t g = u0;
    int trk = u0 < total ? find_track(frame_pfx, T, g) : 0;
    // The wave-cooperative path: when every lane of the wave owns a whole run of RUN frames of one
    // track, the runs 16-B aligned and their whole sample streams inside the track (every step is
    // the plain step below), each step's 32 samples per lane come in by 8 loads per wave that each
    // read the 128-byte segments of 8 lanes (8 cache lines per load instead of 64: a lane's own
    // 16-B loads of its segment each hit a different line than the other lanes'), through a
    // per-wave LDS tile.  The folds are the plain step's, so the values are identical.
    {
        const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
        bool ok = u0 < total && u1 - u0 == (uint64_t)RUN && u1 <= frame_pfx[trk + 1];
        uint64_t f0 = 0, a0 = 0, n = 0;
        if (ok) {
            f0 = g - frame_pfx[trk];
            n = n_len[trk];
            a0 = src_off[trk] + f0 * (uint64_t)hop;
            ok = (a0 & 3u) == 0 && f0 * (uint64_t)hop + (uint64_t)(RUN + G - 1) * (uint64_t)hop <= n;
        }
        const int trk0 = __builtin_amdgcn_readfirstlane(trk);
        if (__builtin_amdgcn_ballot_w64(!(ok && trk == trk0)) == 0) {
            const f4* q = reinterpret_cast<const f4*>(x);
            const uint64_t blkw = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a0 >> 2)) |
                                   ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a0 >> 34)) << 32));
            const uint64_t bstride = (uint64_t)RUN * (uint64_t)hop / 4;  // blocks between lanes' runs
            const uint64_t lbase = blkw + (uint64_t)(l >> 3) * bstride + (uint64_t)(l & 7);
            const float gn = gain[trk];
            const int nseg = RUN + G - 1, spseg = hop >> 5, steps = nseg * spseg;
            f4 stg[8];
            auto issue = [&](int t) {
#pragma unroll
                for (int k = 0; k < 8; k++) stg[k] = q[lbase + (uint64_t)(8 * k) * bstride + 8 * (uint64_t)t];
            };
            auto wave_sync = [] {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            };
            float acc[G];
#pragma unroll
            for (int r = 0; r < G; r++) acc[r] = 0.0f;
            issue(0);
            int t = 0;
            for (int sg = 0; sg <= nseg; sg++) {
#pragma unroll
                for (int r = 0; r < G; r++) {
                    if (sg % G != r) continue;  // wave-uniform
                    if (sg >= G) {              // frame sg - G (< RUN) of the run: whole, inside the track
                        const uint64_t fj = f0 + (uint64_t)(sg - G);
                        rms[frame_pfx[trk] + fj] = __builtin_sqrtf(acc[r] / (float)fs);
                    }
                    acc[r] = 0.0f;
                }
                if (sg == nseg) break;
                for (int c = 0; c < spseg; c++, t++) {
                    wave_sync();  // the previous step's tile reads are done
#pragma unroll
                    for (int k = 0; k < 8; k++) tile[wv][8 * k + (l >> 3)][l & 7] = stg[k];
                    wave_sync();
                    f4 cur[8];
#pragma unroll
                    for (int e = 0; e < 8; e++) cur[e] = tile[wv][l][e];
                    if (t + 1 < steps) issue(t + 1);
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const float v[4] = {cur[e].x, cur[e].y, cur[e].z, cur[e].w};
#pragma unroll
                        for (int w = 0; w < 4; w++) {
                            const float y = v[w] * gn;
                            const float yy = y * y;
#pragma unroll
                            for (int r = 0; r < G; r++) acc[r] += yy;
                        }
                    }
                }
            }
            return;
        }
    }
    if (u0 >= total) return;
    while (g < u1) {  // one piece per track the run touches
        while (g >= frame_pfx[trk + 1]) trk++;
        const uint64_t f0 = g - frame_pfx[trk];
        const uint64_t gend = u1 < frame_pfx[trk + 1] ? u1 : frame_pfx[trk + 1];
        const int nf = (int)(gend - g);
        const uint64_t n = n_len[trk];
        const uint64_t s0 = f0 * (uint64_t)hop;  // the piece's first sample (track-relative)
        const uint64_t a0 = src_off[trk] + s0;   // its float index in x
        const int d = (int)(a0 & 3u);
        const uint64_t blk0 = (a0 - (uint64_t)d) >> 2;
        const uint64_t last = (src_off[trk] + (n > 0 ? n - 1 : 0)) >> 2;  // last block holding a sample
        const int64_t ls = (int64_t)(n - s0);                               // samples left in the track
        const f4* q = reinterpret_cast<const f4*>(x);
        const float gn = gain[trk];
        float acc[G];
#pragma unroll
        for (int r = 0; r < G; r++) acc[r] = 0.0f;
        auto load = [&](uint64_t bi) { return q[bi < last ? bi : last]; };
        // the piece's samples as one stream of 16-B blocks (stream position p of block element e:
        // 4 (block - blk0) + e - d), 8 blocks per step with the next 8 in flight; every hop / 32
        // steps a segment ends: frame sg - G is stored and frame sg starts in its accumulator
        const int nseg = nf + G - 1;
        const int spseg = hop >> 5;  // 8-block steps per segment
        f4 buf[9];
#pragma unroll
        for (int e = 0; e < 9; e++) buf[e] = load(blk0 + (uint64_t)e);
        uint64_t bi = blk0 + 9;
        for (int sg = 0; sg <= nseg; sg++) {
#pragma unroll
            for (int r = 0; r < G; r++) {
                if (sg % G != r) continue;  // wave-uniform
                if (sg >= G && sg - G < nf) {
                    const uint64_t fj = f0 + (uint64_t)(sg - G);
                    const uint64_t st = fj * (uint64_t)hop;
                    const uint64_t en = st + (uint64_t)fs < n ? st + (uint64_t)fs : n;
                    const int len = en > st ? (int)(en - st) : 0;
                    rms[frame_pfx[trk] + fj] = len > 0 ? __builtin_sqrtf(acc[r] / (float)len) : 0.0f;
                }
                acc[r] = 0.0f;
            }
            if (sg == nseg) break;
            const int64_t p0 = (int64_t)sg * hop;
            if (p0 >= ls) continue;  // past the track: every remaining term is +0
            for (int c = 0; c < spseg; c++) {
                f4 nb[8];
#pragma unroll
                for (int e = 0; e < 8; e++) nb[e] = load(bi + (uint64_t)e);
                // the common step: 16-B aligned piece, all 32 samples inside the track, on every
                // lane of the wave: the samples are the blocks' own components, no selects
                const bool plain = d == 0 && p0 + 32 * (c + 1) <= ls;
                if (__builtin_expect(__builtin_amdgcn_ballot_w64(!plain) == 0, 1)) {
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const float v[4] = {buf[e].x, buf[e].y, buf[e].z, buf[e].w};
#pragma unroll
                        for (int w = 0; w < 4; w++) {
                            const float y = v[w] * gn;
                            const float yy = y * y;
#pragma unroll
                            for (int t = 0; t < G; t++) acc[t] += yy;
                        }
                    }
                    buf[0] = buf[8];
#pragma unroll
                    for (int e = 0; e < 8; e++) buf[e + 1] = nb[e];
                    bi += 8;
                    continue;
                }
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    const f4 cur = buf[e], nxt = buf[e + 1];
                    float v[4];
                    v[0] = d == 0 ? cur.x : d == 1 ? cur.y : d == 2 ? cur.z : cur.w;
                    v[1] = d == 0 ? cur.y : d == 1 ? cur.z : d == 2 ? cur.w : nxt.x;
                    v[2] = d == 0 ? cur.z : d == 1 ? cur.w : d == 2 ? nxt.x : nxt.y;
                    v[3] = d == 0 ? cur.w : d == 1 ? nxt.x : d == 2 ? nxt.y : nxt.z;
                    const int64_t pk = p0 + 32 * c + 4 * e;
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        const float y = (pk + w < ls ? v[w] : 0.0f) * gn;
                        const float yy = y * y;
#pragma unroll
                        for (int t = 0; t < G; t++) acc[t] += yy;
                    }
                }
                buf[0] = buf[8];
#pragma unroll
                for (int e = 0; e < 8; e++) buf[e + 1] = nb[e];
                bi += 8;
            }
        }
        g = gend;
    }
}

void launch_frame_rms(const float* x, const uint64_t* src_off, const float* gain, const uint64_t* n_len,
                      const uint64_t* frame_pfx, int T, uint64_t total, int fs, int hop, float* rms, hipStream_t st,
                      bool per_frame_kernel) {
    if (total == 0) return;
    const bool per_frame = per_frame_kernel;  // the debug probe selects the per-frame kernel
    const int G = hop > 0 && fs % hop == 0 ? fs / hop : 0;
    if (!per_frame && hop % 32 == 0 && (G == 1 || G == 2 || G == 4 || G == 8)) {
        const uint64_t per_wg = 256 * 4 * (uint64_t)G;  // frames per workgroup: 256 lanes x RUN
        const dim3 grid((unsigned)((total + per_wg - 1) / per_wg));
        if (G == 1)
            hipLaunchKernelGGL(k_frame_rms_run<1>, grid, dim3(256), 0, st, x, src_off, gain, n_len, frame_pfx, T, total, fs, hop, rms);
        else if (G == 2)
            hipLaunchKernelGGL(k_frame_rms_run<2>, grid, dim3(256), 0, st, x, src_off, gain, n_len, frame_pfx, T, total, fs, hop, rms);
        else if (G == 4)
            hipLaunchKernelGGL(k_frame_rms_run<4>, grid, dim3(256), 0, st, x, src_off, gain, n_len, frame_pfx, T, total, fs, hop, rms);
        else
            hipLaunchKernelGGL(k_frame_rms_run<8>, grid, dim3(256), 0, st, x, src_off, gain, n_len, frame_pfx, T, total, fs, hop, rms);
        return;
    }
    hipLaunchKernelGGL(k_frame_rms, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, src_off, gain, n_len,
                       frame_pfx, T, total, fs, hop, rms, 0);
}

// The energy pass's frame RMS from the trim pass's (one read of the samples for both): with the
// trim pass run on the raw signal at the energy hop, and every trim start a multiple of that hop
// (trim frames start at multiples of fs / 2, a multiple of hop), trimmed frame j of track i is
// raw frame raw_base[i] + j whenever it is whole (j hop + fs <= n_trim): the same samples, gain
// and fold order, so the same value.  Frames cut short by the trimmed end are folded again by
// k_frame_rms (only_partial).
__global__ __launch_bounds__(256) void k_rms_gather(const float* __restrict__ raw, const uint64_t* __restrict__ raw_base,
                                                    const uint64_t* __restrict__ frame_pfx, int T, uint64_t total,
                                                    const uint64_t* __restrict__ n_trim, int fs, int hop,
                                                    float* __restrict__ rms) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const int i = find_track(frame_pfx, T, g);
    const uint64_t j = g - frame_pfx[i];
    if (j * (uint64_t)hop + (uint64_t)fs <= n_trim[i]) rms[g] = raw[raw_base[i] + j];
}
void launch_frame_rms_from_raw(const float* raw, const uint64_t* raw_base, const float* x, const uint64_t* src_off,
                               const float* gain, const uint64_t* n_trim, const uint64_t* frame_pfx, int T, uint64_t total,
                               int fs, int hop, float* rms, hipStream_t st) {
    if (total == 0) return;
    const dim3 grid((unsigned)((total + 255) / 256));
    hipLaunchKernelGGL(k_rms_gather, grid, dim3(256), 0, st, raw, raw_base, frame_pfx, T, total, n_trim, fs, hop, rms);
    hipLaunchKernelGGL(k_frame_rms, grid, dim3(256), 0, st, x, src_off, gain, n_trim, frame_pfx, T, total, fs, hop, rms, 1);
}
void launch_trim(const float* rms, const uint64_t* frame_pfx, int T, const uint64_t* n_raw, int hop, float thr,
                 uint64_t min_frames, int enable, uint64_t* trim_start, uint64_t* trim_end, hipStream_t st,
                 const uint64_t* base_pfx, int stride) {
    if (T == 0) return;
    hipLaunchKernelGGL(k_trim, dim3(T), dim3(256), 0, st, rms, frame_pfx, base_pfx ? base_pfx : frame_pfx,
                       base_pfx ? stride : 1, T, n_raw, hop, thr, min_frames, enable, trim_start, trim_end);
}
void launch_energy_onsets(const float* rms, const uint64_t* frame_pfx, const uint64_t* n_trim, int hop, float factor,
                          uint32_t* out, const uint64_t* out_off, int* out_n, int T, hipStream_t st) {
    if (T == 0) return;
    hipLaunchKernelGGL(k_energy_onsets, dim3(T), dim3(256), 0, st, rms, frame_pfx, n_trim, hop, factor, out, out_off,
                       out_n);
}
void launch_flux_onsets(const float* sfo, const float* hfc, const float* hpe, float* scratch, const uint64_t* frame_pfx,
                        const uint64_t* n_trim, int hop, float pct, uint32_t* out, const uint64_t* out_off,
                        int* out_n, int T, hipStream_t st) {
    if (T == 0) return;
    const int kinds = hpe ? 3 : 2;
    hipLaunchKernelGGL(k_flux_onsets, dim3(kinds * T), dim3(256), 0, st, sfo, hfc, hpe, scratch, frame_pfx, n_trim, hop,
                       pct, out, out_off, out_n, T);
}
void launch_consensus(const uint32_t* energy, const uint64_t* e_off, const int* e_n, const uint32_t* flux_on,
                      const uint64_t* f_off, const int* f_n, uint64_t kind_stride, int T, uint32_t tol, int enable,
                      const int* has_mags, uint32_t* chosen, const uint64_t* c_off, int* c_n, uint32_t* scratch,
                      hipStream_t st, int hpss) {
    if (T == 0) return;
    hipLaunchKernelGGL(k_consensus, dim3(T), dim3(256), 0, st, energy, e_off, e_n, flux_on, f_off, f_n, kind_stride, T,
                       tol, enable, has_mags, chosen, c_off, c_n, scratch, hpss);
}

}  // namespace sdsp
