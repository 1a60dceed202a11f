// k_features.hip — every per-frame reduction of the 2048-point magnitude spectrogram in one
// pass over HBM (reference src/features/period/novelty.rs and src/features/onset/*):
//
//   E[v][t]   = sum_k |X_t[k]|^2 over band v          energy_flux_novelty(_band)  novelty.rs:504-508,641-644
//   H[v][t]   = sum_k (k*|X_t[k]|)*|X_t[k]|           hfc_novelty(_band) / detect_hfc_onsets  :738-747,810-821, hfc.rs:130-137
//   SFX[v][t] = sqrt(sum_k max(0, L_t[k] - max_{|j-k|<=K, j in band} L_{t-1}[j])^2)   superflux(_band) :353-376,419-442
//   SFO[t]    = sqrt(sum_k max(0, X_t[k]/max_t - X_{t-1}[k]/max_{t-1})^2)            spectral_flux.rs:116-157
//   MEL[m][t] = sum_k L_t[k] * w_{k,m}  (HTK triangles, bins ascending)               MelFilterbank::apply_logmag :174-190
//   with L = ln(1 + max(X, 0)), v in {full, low, mid, high}.
//
// Each workgroup owns FT_STEP consecutive frames of one track, one thread per frame, so
// every per-frame fold runs in exactly the reference's bin order (bit-identical to the CPU
// restatement).  Each wave covers 63 frames in lanes 1-63; lane 0 is a helper holding the frame
// before the wave's first.  The spectral flux needs X/max of every frame twice (as frame t and as
// frame t-1 of the next); each lane divides its own frame's bins once and takes the previous
// frame's quotients from lane - 1 (DPP wave shift), halving the per-bin IEEE divisions.  Bins
// are streamed through two circular LDS windows of W columns (slot = bin mod W): raw magnitudes
// and their logs.  Each wave stages the 64 rows of its own lanes (no workgroup barrier in the
// walk).  Each step loads the CW bins K ahead of the ones it processes (row segments, log
// computed once per element from a two-column table, sd_logf_ge1_t2), so the SuperFlux max
// filter over [b-K, b+K] of the previous frame always finds its halo resident and no column is
// loaded or logged twice.  Row stride W+1 (odd) keeps the per-thread row walks
// bank-conflict-free.
//
// Mel bands: every bin feeds at most two adjacent triangles (or one narrow triangle twice,
// rising then falling edge) and the triangles start in bin order, so a thread keeps only two
// running sums (mels mA, mA+1) in registers; the host precomputes, per bin, how many
// finished mels to flush before the bin (uniform across the workgroup) and the ordered
// (accumulator, weight) contributions.  Flushed mels are stored mel-major (MEL[m*total + t]),
// coalesced across the workgroup.  Within the mel range the 8 plans of a chunk are packed
// (MelChunk) and read with one scalar load.
#include <stdexcept>
#include <type_traits>

#include "kernels.hpp"

namespace sdsp {



// the per-chunk tables (flags, packed mel plans, HFC weights) through the constant address space:
// the kernel never writes them, so they come in by scalar loads into SGPRs (through a generic
// pointer the compiler cannot prove that and loads them per lane, then reads the first lane)
typedef const __attribute__((address_space(4))) int* ConstI;
typedef const __attribute__((address_space(4))) MelChunk* ConstMC;

// KK > 0: compile-time SuperFlux half width (the default 4) -- the previous frame's logs for
// the chunk's windows are read once into registers and every bin's window max is taken from
// them; KK = 0: runtime P.K with the per-bin window loop.
template <int CW, int W, int KK>
__global__ __launch_bounds__(FT_FRAMES) __attribute__((amdgpu_waves_per_eu(KK > 0 ? 3 : 1))) void k_features(const RowMap rm,
                                                        const uint64_t* __restrict__ frame_pfx,
                                                        const uint64_t* __restrict__ tile_pfx, int T, FeatParams P,
                                                        const MelPlan* __restrict__ mel, float* __restrict__ E,
                                                        float* __restrict__ H, float* __restrict__ SFX,
                                                        float* __restrict__ SFO, float* __restrict__ MEL,
                                                        uint64_t total) {
    static_assert((W & (W - 1)) == 0, "W must be a power of two");
    constexpr int ROWS = FT_FRAMES;  // row i: lane i's frame (each wave stages its own 64 rows)
    constexpr int LS = W + 1;
    // slot s of row r: {magnitude, ln(1 + max(magnitude, 0))} side by side, so the walk reads both
    // with one ds_read_b64 at a per-chunk base plus an immediate offset (the chunk's 8 slots never
    // wrap: CW divides W), and the staging writes both with one ds_write_b64
    __shared__ float2 ML[ROWS][LS];
    // the staging's log tables (sd_ln1p_x_t9_finite): {s, ln c} per 9-bit mantissa index and
    // {e LN2_HI, RN(e LN2_LO)} per exponent, read per element
    __shared__ sd_logtab2_t ltab[512];
    __shared__ sd_ln2tab_t etab[129];
    static_assert(KK == 0 || CW + 2 * KK <= W, "window halo must fit the ring");
    for (int q = threadIdx.x; q < 512; q += FT_FRAMES) ltab[q] = SD_LOGTAB9_D[q];
    for (int q = threadIdx.x; q < 129; q += FT_FRAMES) etab[q] = sd_ln2tab_from(q);

    const uint64_t gb = blockIdx.x;
    const int trk = find_track(tile_pfx, T, gb);
    const int64_t F = (int64_t)(frame_pfx[trk + 1] - frame_pfx[trk]);
    const int64_t f0 = (int64_t)(gb - tile_pfx[trk]) * FT_STEP;
    const uint64_t g0 = frame_pfx[trk];
    const int i = threadIdx.x;
    const bool helper = (i & 63) == 0;
    const int ro = i;  // this lane's LDS row
    const int64_t f = f0 - 1 + 63 * (i >> 6) + (i & 63);
    const bool own_ok = f >= 0 && f < F;
    const bool valid = !helper && f < F;  // ro >= 1 here, so f >= 0
    const bool has_prev = valid && f >= 1;
    const int K = KK > 0 ? KK : P.K, B = P.B;
    const uint64_t g = g0 + (uint64_t)f;

    float e[4] = {0, 0, 0, 0}, h[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0}, so = 0.0f;
    // The sub-bands are disjoint and ascend in bin order (pipeline: low [b0, bl), mid [bl, bm),
    // high [bm, bh)), so each band's folds are one contiguous run of the walk: they go to the
    // accumulators eb/hb/sb of the band the walk is in (cur, wave-uniform), which are stored
    // into e/h/sx[cur] when the run ends.  Per bin that is one add each instead of a select per
    // band, and the band's SuperFlux term is the full band's (same product) except within K
    // bins of a band edge.
    float eb = 0.0f, hb = 0.0f, sb = 0.0f;
    int cur = 0;
    auto band_of = [&](int b) {
        int v = 0;
#pragma unroll
        for (int q = 3; q >= 1; q--)
            if (P.band_on[q] && b >= P.bs[q] && b < P.be[q]) v = q;
        return v;
    };
    auto flush = [&]() {
        if (cur == 1) e[1] = eb, h[1] = hb, sx[1] = sb;
        else if (cur == 2) e[2] = eb, h[2] = hb, sx[2] = sb;
        else if (cur == 3) e[3] = eb, h[3] = hb, sx[3] = sb;
        eb = hb = sb = 0.0f;
    };
    float accA = 0.0f, accB = 0.0f;
    int mA = 0;
    float* melA = MEL;  // MEL row mA (wave-uniform, advanced with mA)
    // MEL row mA as a buffer resource of `total` floats; lanes without a frame get an offset past
    // it, so their stores are dropped (no exec-mask branch per flush)
    const uint32_t mel_vo = valid ? (uint32_t)g * 4u : 0xFFFFFFF0u;
    auto mel_rsrc = [&]() {
        return __builtin_amdgcn_make_buffer_rsrc((void*)melA, (short)0, (int)(uint32_t)(total * 4u), 0x00020000);
    };
    // frame f of this track lives in row (f even ? A : B) r0 + (f >> 1) * step (RowMap)
    const uint64_t ra0 = rm.rowA0[trk], rb0 = rm.rowB0 ? rm.rowB0[trk] : ra0 + (uint64_t)rm.offB;
    auto row_of = [&](int64_t fr, bool* odd) {
        *odd = fr & 1;
        return (*odd ? rb0 + (uint64_t)(fr >> 1) * (uint64_t)rm.stepB : ra0 + (uint64_t)(fr >> 1) * (uint64_t)rm.stepA);
    };
    auto fmax_of = [&](int64_t fr) {
        bool odd;
        const uint64_t r = row_of(fr, &odd);
        return odd ? rm.fmaxB[r] : rm.fmaxA[r];
    };
    const float mx_c = own_ok ? fmax_of(f) : 0.0f;
    const bool cn = mx_c > EPS;
    // X / max by one correctly rounded reciprocal per frame and an FMA correction per bin:
    // q0 = m yr, q = q0 + (m - max q0) yr is the correctly rounded m / max for normal operands whose
    // quotient and residual stay normal (tools/check_div_fast.hip: all 2^46 mantissa pairs, and
    // v_rcp-free here: yr is an IEEE division).  That holds for m = 0 and m in [max 2^-120, inf)
    // with m >= 2^-100 and max <= 2^100; cn = false gives yr = 0, so q = 0 as the reference's
    // zeroed frame.  A chunk where some lane of the wave saw another m redoes its flux terms with
    // the IEEE division (rare: needs magnitudes 2^-100 below the frame maximum, or inf / NaN).
    const float yr = cn ? 1.0f / mx_c : 0.0f;
    const bool q_frame_ok = !cn || mx_c <= 0x1p100f;
    const uint32_t q_lim = __float_as_uint(sd_maxf(0x1p-100f, mx_c * 0x1p-120f)) - 1u;
    uint32_t q_lo = 0xFFFFFFFFu, q_hi = 0u;  // min of bits(m) - 1, max of bits(m) over the chunk
    auto quot = [&](float m) {
        const uint32_t u = __float_as_uint(m);
        q_lo = min(q_lo, u - 1u);
        q_hi = max(q_hi, u);
        const float q0 = m * yr;
        return __builtin_fmaf(__builtin_fmaf(-mx_c, q0, m), yr, q0);
    };
    // the chunk's flux terms again with the IEEE division, from the fold's value at the chunk
    // start, when some lane's quotient left the exact range
    auto quot_redo = [&](int c0, int nb, float so_start) {
        const bool miss = !q_frame_ok || q_lo < q_lim || q_hi >= 0x7F800000u;
        q_lo = 0xFFFFFFFFu;
        q_hi = 0u;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(miss) == 0, 1)) return;
        so = so_start;
        for (int j = 0; j < nb; j++) {
            const float m = ML[ro][(c0 + j) & (W - 1)].x;
            const float cv = cn ? m / mx_c : 0.0f;
            const float pv = __builtin_bit_cast(
                float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, cv), 0x138, 0xf, 0xf, true));
            const float d = max_bnn(cv - pv, 0.0f);
            so += d * d;
        }
    };

    // Each wave stages the rows of its own 64 lanes (frames f0 - 1 + 63 w + l), so the waves
    // share no LDS row and run without workgroup barriers: a wave's LDS operations execute in
    // issue order, and a compiler barrier keeps the staging writes and the walk's reads in
    // program order.  (The helper row duplicates the previous wave's last row: 1/64 extra loads.)
    const int lane = i & 63, wrow = i & ~63;
    const int sub = lane / CW, jj = lane % CW;
    const int64_t fw = f0 - 1 + 63 * (i >> 6);  // frame of the wave's row 0

    // stage bins [b0, b0+CW) (columns beyond B or rows outside the track read as 0); the loads
    // of the next step are in flight while the current step is walked
    constexpr int RSTEP = 64 / CW;
    constexpr int NLD = CW;
    const float* rowp[NLD];  // this thread's staged rows
#pragma unroll
    for (int u = 0; u < NLD; u++) {
        const int64_t fr = fw + sub + u * RSTEP;
        rowp[u] = rm.magsA;  // rows outside the track: a valid address, the value is replaced by 0
        if (fr >= 0 && fr < F) {
            bool odd;
            const uint64_t row = row_of(fr, &odd);
            rowp[u] = (odd ? rm.magsB : rm.magsA) + row * (uint64_t)P.stride;
        }
    }
    float nx[NLD];
    // unconditional loads (the zeros are selected afterwards): no branch per load, so the
    // compiler's wait counts stay per load (1.5 % faster than guarded loads; a second chunk in
    // flight measured no faster, so load latency is not what bounds the kernel)
    uint32_t row_ok = 0;
#pragma unroll
    for (int u = 0; u < NLD; u++) {
        const int64_t fr = fw + sub + u * RSTEP;
        row_ok |= (uint32_t)(fr >= 0 && fr < F) << u;
    }
    auto load = [&](int b0) {
        const int b = b0 + jj;
        const int bc = b < B ? b : B - 1;
#pragma unroll
        for (int u = 0; u < NLD; u++) nx[u] = rowp[u][bc];
    };
    auto fix = [&](int b0) {  // zeros for columns past B and rows outside the track
        const bool col_ok = b0 + jj < B;
        // only a track's last tile has rows outside it, and only the last chunks columns past B:
        // a wave with neither skips the selects
        if (__builtin_amdgcn_ballot_w64(!col_ok || row_ok != (1u << NLD) - 1u) == 0) return;
#pragma unroll
        for (int u = 0; u < NLD; u++) nx[u] = (col_ok && ((row_ok >> u) & 1)) ? nx[u] : 0.0f;
    };
    auto commit = [&](int b0) {
        fix(b0);
        const int slot = (b0 + jj) & (W - 1);
#pragma unroll
        for (int u = 0; u < NLD; u++) {
            const int r = wrow + sub + u * RSTEP;
            // sd_ln1p_max0_t2 with the max taken by max0_quiet (the staged magnitudes are
            // arithmetic results or zeros, never signalling NaNs) and the 9-bit-table, degree-4
            // evaluation, bit-identical to sd_logf on every finite f32 >= 1 (sdsp_libm.h)
            const float xx = 1.0f + max0_quiet(nx[u]);
            const float lv = sd_ln1p_x_t9_finite(xx, ltab, etab);
            ML[r][slot] = make_float2(nx[u], xx < SD_INF_F ? lv : xx);
        }
    };
    __syncthreads();  // ltab; from here on each wave works on its own rows
    // prologue: bins [0, K) (K <= CW); the ring slots of bins [-K, 0) read as L = 0
    if (jj < K) {
        load(0);
        commit(0);
    }
    if (KK > 0)
        for (int q = 0; q < KK; q++) ML[ro][W - KK + q].y = 0.0f;
    load(K);
    for (int c0 = 0; c0 < B; c0 += CW) {
        // the wave's walk of the previous step has issued its reads of the slots overwritten here
        asm volatile("" ::: "memory");
        commit(c0 + K);
        asm volatile("" ::: "memory");
        if (c0 + CW < B) load(c0 + CW + K);
        const int nb = B - c0 < CW ? B - c0 : CW;
        // a wave with no valid frame skips the walk; lanes of invalid frames in a partly valid
        // wave walk zero rows (their results are not stored), which keeps the band bookkeeping
        // (cur) wave-uniform
        if (__builtin_amdgcn_ballot_w64(valid) == 0) continue;
        // KK > 0: previous frame's L for bins [c0 - KK, c0 + CW + KK) (0 outside [0, B))
        float Rw[KK > 0 ? CW + 2 * KK : 1];
        // with 2 KK = CW, the window maxima over [j, j + 2 KK] of Rw, j < CW, split at CW into a
        // suffix max of Rw[j..CW) and a prefix max of Rw[CW..j+2KK] (exact: max is a selection,
        // and every L >= +0): 3 CW - 2 max operations instead of 2 KK CW
        constexpr bool VHK = KK > 0 && 2 * KK == CW;
        float Wm[VHK ? CW : 1];
        // every lane walks the flux terms (no divergent branch per bin); lanes without a previous
        // frame read row max(ro - 1, 0) and their sums are never stored
        const int rp = lane > 0 ? ro - 1 : ro;
        if (KK > 0) {
#pragma unroll
            for (int q = 0; q < (KK > 0 ? CW + 2 * KK : 1); q++) Rw[q] = ML[rp][(c0 - KK + q) & (W - 1)].y;
            if constexpr (VHK) {
                float suf[CW], pre[CW];
                suf[CW - 1] = Rw[CW - 1];
#pragma unroll
                for (int q = CW - 2; q >= 0; q--) suf[q] = max_bnn(Rw[q], suf[q + 1]);
                pre[0] = Rw[CW];
#pragma unroll
                for (int q = 1; q < CW; q++) pre[q] = max_bnn(pre[q - 1], Rw[CW + q]);
#pragma unroll
                for (int q = 0; q < CW; q++) Wm[q] = max_bnn(suf[q], pre[q]);
            }
        }
        if constexpr (VHK) {
            // fast chunk (most bins: above the mel and sub-band ranges, or inside one band away
            // from its edges): the same per-bin arithmetic with the band and mel bookkeeping
            // hoisted to the chunk, so the walk issues no scalar work per bin; a mel chunk
            // (FT_CHUNK_MEL, the 30-8000 Hz range) adds the mel sums from the chunk's packed plan
            // (7.63 -> 7.17 ms per launch against the general walk for those chunks)
            const int cf = ((ConstI)P.chunk_flags)[c0 / CW];
            if (cf & (FT_CHUNK_FAST | FT_CHUNK_MEL)) {
                const int vbc = cf & 3;
                if (vbc != cur) {
                    flush();
                    cur = vbc;
                }
                const float so_start = so;
                // MEL: the chunk's mel plans come in one scalar load; a flush stores accA through a
                // buffer resource whose record count drops the stores of lanes without a frame
                // NOBAND: a chunk outside every sub-band (vbc = 0: most of the bins above the high
                // band's edge), whose walk drops the sub-band folds instead of computing and
                // discarding them (-0.7 % per launch, profiles/r06_kernel_ab_features_noband.txt)
                auto walk = [&](auto mel_tag, auto reg_tag, auto noband_tag) {
                    constexpr bool MEL = decltype(mel_tag)::value;
                    constexpr bool REG = decltype(reg_tag)::value;
                    constexpr bool NOBAND = decltype(noband_tag)::value;
                    MelChunk mc{};
                    const ConstMC mcp = (ConstMC)P.mel_chunks + c0 / CW;
                    if constexpr (MEL) {
                        mc.bits = mcp->bits;
#pragma unroll
                        for (int j = 0; j < CW; j++) mc.w0[j] = mcp->w0[j], mc.w1[j] = mcp->w1[j];
                    }
                    // (float) b from the chunk's scalar-loaded weights: no conversion per bin
                    float bfv[CW];
#pragma unroll
                    for (int j = 0; j < CW; j++) bfv[j] = mcp->bf[j];
#pragma unroll
                    for (int j = 0; j < CW; j++) {
                        const int b = c0 + j;
                        const int s = b & (W - 1);
                        const float2 ml = ML[ro][s];
                        const float m = ml.x;
                        const float ee = m * m;
                        const float hh = bfv[j] * m * m;
                        e[0] += ee;
                        h[0] += hh;
                        const float lc = ml.y;
                        const float cv = quot(m);
                        const float pv = __builtin_bit_cast(
                            float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, cv), 0x138, 0xf, 0xf, true));
                        const float d = max_bnn(cv - pv, 0.0f);
                        so += d * d;
                        const float df = max_bnn(lc - Wm[j], 0.0f);
                        const float df2 = df * df;
                        sx[0] += df2;
                        if (!NOBAND && vbc) {
                            eb += ee;
                            hb += hh;
                            sb += df2;
                        }
                        if constexpr (MEL) {
                            const uint32_t pb = mc.bits >> (4 * j);
                            for (uint32_t q = pb & 3; q > 0; q--) {
                                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(accA), mel_rsrc(), mel_vo, 0, 0);
                                accA = accB;
                                accB = 0.0f;
                                mA++;
                                melA += total;
                            }
                            // as the general walk: L >= +0, so w = 0 terms are skipped, not added
                            // (L = +inf would make them NaN).  REG (FT_CHUNK_MELREG): w0 goes to
                            // accA and w1 to accB on every bin of the chunk, no accumulator select
                            if constexpr (REG) {
                                if (__float_as_uint(mc.w0[j]) << 1) accA += lc * mc.w0[j];
                                if (__float_as_uint(mc.w1[j]) << 1) accB += lc * mc.w1[j];
                            } else if (mc.w0[j] != 0.0f) {
                                if (pb & 4) accB += lc * mc.w0[j];
                                else accA += lc * mc.w0[j];
                            }
                            if (!REG && mc.w1[j] != 0.0f) {
                                if (pb & 8) accB += lc * mc.w1[j];
                                else accA += lc * mc.w1[j];
                            }
                        }
                    }
                };
                if (cf & FT_CHUNK_MELREG)
                    walk(std::true_type{}, std::true_type{}, std::false_type{});
                else if (cf & FT_CHUNK_MEL)
                    walk(std::true_type{}, std::false_type{}, std::false_type{});
                else if (vbc == 0)
                    walk(std::false_type{}, std::false_type{}, std::true_type{});
                else
                    walk(std::false_type{}, std::false_type{}, std::false_type{});
                quot_redo(c0, CW, so_start);
                continue;
            }
        }
        // unrolled (Wm / Rw are register windows indexed by j); the chunk's valid bins are a guard,
        // not an early exit, so the unroll is complete
        const float so_start = so;
#pragma unroll
        for (int j = 0; j < CW; j++) {
            if (j >= nb) continue;
            const int b = c0 + j;
            const int s = b & (W - 1);
            const float2 ml = ML[ro][s];
            const float m = ml.x;
            const float ee = m * m;
            const float hh = (float)b * m * m;
            e[0] += ee;
            h[0] += hh;
            const int vb = band_of(b);
            if (vb != cur) {
                flush();
                cur = vb;
            }
            if (vb) {
                eb += ee;
                hb += hh;
            }
            const float lc = ml.y;
            // X/max of this lane's frame, and of the previous frame from lane - 1 (its frame is
            // f - 1 for every lane that reads it: lanes 1-63; the helper's value is unused)
            const float cv = quot(m);
            const float pv = __builtin_bit_cast(
                float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, cv), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
            if (P.n_mels > 0) {
                const MelPlan mp = mel[b];
                for (int q = 0; q < mp.nflush; q++) {
                    if (valid) MEL[(uint64_t)mA * total + g] = accA;
                    accA = accB;
                    accB = 0.0f;
                    mA++;
                    melA += total;
                }
                // novelty.rs:181-186 skips v <= 0.  Here v = lc >= +0 always (sd_maxf maps NaN to 0,
                // as f32::max), so the skipped terms are +0 * w = +0, and adding +0 to a
                // non-negative sum is exact: no per-lane branch
                if (mp.w0 != 0.0f) {
                    if (mp.s0 == 0) accA += lc * mp.w0;
                    else accB += lc * mp.w0;
                }
                if (mp.w1 != 0.0f) {
                    if (mp.s1 == 0) accA += lc * mp.w1;
                    else accB += lc * mp.w1;
                }
            }
            {
                const float d = max_bnn(cv - pv, 0.0f);
                so += d * d;
                // SuperFlux, full band window [b-K, b+K] clipped to [0, B).  Every L >= +0 and
                // max is an exact selection, so the max over the register window (entries
                // outside [0, B) are +0) equals the reference's max from 0 over the clipped range.
                const int lo = b - K < 0 ? 0 : b - K;
                const int hi = b + K + 1 < B ? b + K + 1 : B;
                float pm = 0.0f;
                if constexpr (KK > 0) {
                    if constexpr (VHK) {
                        pm = Wm[j];
                    } else {
                        pm = Rw[j];
#pragma unroll
                        for (int q = 1; q <= 2 * KK; q++) pm = max_bnn(pm, Rw[j + q]);
                    }
                } else {
                    for (int q = lo; q < hi; q++) pm = max_bnn(pm, ML[rp][q & (W - 1)].y);  // L is never NaN
                }
                const float df = max_bnn(lc - pm, 0.0f);
                const float df2 = df * df;
                sx[0] += df2;
                if (vb) {
                    const int bsv = P.bs[vb], bev = P.be[vb];
                    if (lo < bsv || hi > bev) {  // window clipped at the band edge
                        const int lb = lo < bsv ? bsv : lo;
                        const int hbd = hi > bev ? bev : hi;
                        float pmb = 0.0f;
                        if constexpr (KK > 0) {
#pragma unroll
                            for (int q = 0; q <= 2 * KK; q++)
                                if (b - KK + q >= lb && b - KK + q < hbd) pmb = max_bnn(pmb, Rw[j + q]);
                        } else {
                            for (int q = lb; q < hbd; q++) pmb = max_bnn(pmb, ML[rp][q & (W - 1)].y);
                        }
                        const float db = max_bnn(lc - pmb, 0.0f);
                        sb += db * db;
                    } else {
                        sb += df2;
                    }
                }
            }
        }
        quot_redo(c0, nb, so_start);
    }
    flush();
    if (!valid) return;
    for (; mA < P.n_mels; mA++) {
        MEL[(uint64_t)mA * total + g] = accA;
        accA = accB;
        accB = 0.0f;
    }
#pragma unroll
    for (int v = 0; v < 4; v++) {
        E[(uint64_t)v * total + g] = e[v];
        H[(uint64_t)v * total + g] = h[v];
    }
    if (has_prev) {
        const uint64_t gp = g - 1;  // pair (t-1, t) stored at t-1
        SFO[gp] = __builtin_sqrtf(so);
#pragma unroll
        for (int v = 0; v < 4; v++) SFX[(uint64_t)v * total + gp] = __builtin_sqrtf(sx[v]);
    }
}

void launch_features(const RowMap& mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx,
                     int T, uint64_t n_tiles, const FeatParams& P, const MelPlan* mel, float* E, float* H, float* SFX,
                     float* SFO, float* MEL, uint64_t total, hipStream_t st) {
    if (n_tiles == 0) return;
    if (total >= (1ull << 30)) throw std::runtime_error("launch_features: too many frames for one launch");  // MEL row resources

    // window must hold [c0-K, c0+CW+K): CW + 2K <= W
    if (P.K == 4)
        hipLaunchKernelGGL((k_features<8, 16, 4>), dim3((unsigned)n_tiles), dim3(FT_FRAMES), 0, st, mags,
                           frame_pfx, tile_pfx, T, P, mel, E, H, SFX, SFO, MEL, total);
    else if (P.K <= 4)
        hipLaunchKernelGGL((k_features<8, 16, 0>), dim3((unsigned)n_tiles), dim3(FT_FRAMES), 0, st, mags,
                           frame_pfx, tile_pfx, T, P, mel, E, H, SFX, SFO, MEL, total);
    else
        hipLaunchKernelGGL((k_features<16, 32, 0>), dim3((unsigned)n_tiles), dim3(FT_FRAMES), 0, st, mags,
                           frame_pfx, tile_pfx, T, P, mel, E, H, SFX, SFO, MEL, total);
}

}  // namespace sdsp
