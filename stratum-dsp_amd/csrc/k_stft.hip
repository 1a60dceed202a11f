// k_stft.hip — batched real-input STFT magnitudes for gfx950 (replaces compute_stft,
// reference src/features/chroma/extractor.rs:301-359, whose FFT is rustfft).
//
// Arithmetic: exactly the STFT section of sdsp_fft_spec.h (Stockham radix-4 DIF stages with FMA
// complex products and no W^0 products, then the real-FFT post-processing in FMA form), so the
// spectra are bit-identical to the CPU restatement.  Data movement: two consecutive radix-4
// stages touch a closed set of 16 elements (stage (n, s) butterflies p = p' + j'*n/16,
// j' = 0..3, feed stage (n/4, 4s) butterflies q + s*jA), so each thread runs both stages on 16
// values held in registers ("radix-16 pass"): one LDS round trip per two stages instead of one
// per stage.
//
//   N = 8192 (M = 4096 = 16^3):       3 radix-16 passes, 256 threads per frame
//   N = 2048 (M = 1024 = 16^2 * 4):   2 radix-16 passes + 1 radix-4 pass, 64 threads (one
//                                     wave) per frame, 4 frames per workgroup
//
// Instruction economy (the kernel is VALU-bound):
//  * complex values are pairs of scalar f32 registers.  gfx950's packed f32 ops (v_pk_*) issue
//    at the same flop rate as scalar ones but add a wait state between dependent packed ops, and
//    the -i rotations / conjugations cost extra moves in packed form; scalar code folds them into
//    the adds.  A complex product is 2 v_mul + 2 v_fma;
//  * the W^0 products the spec omits are skipped at compile time where the twiddle is
//    wave-uniform (the last pass); where it is per lane (lanes with p = 0 in passes 1-2) the
//    per-thread table holds exactly (1, +0), whose FMA product equals the operand;
//  * the frame, the window and the per-thread twiddle tables are read with buffer loads
//    whose per-element offsets are scalar (SGPR) constants, so no VALU address arithmetic;
//  * every LDS index is (per-thread base) + (compile-time constant);
//  * bins k and M-k share one LDS read and one S/D evaluation; |X| uses the exact fast sqrt.
// The twiddle values are those of sdsp_fft_spec.h, re-laid out per thread on the host
// (stft_tables below).  LDS index padding i + i/16 keeps the strided pass-1 stores
// near conflict-free.
//
// Ragged batches: the flat frame index (frame_pfx prefix sums) picks the track.  Frames are
// numbered XCD-contiguously (xcd_block) so the 16x (N=8192) / 4x (N=2048) overlap between
// neighbouring frames is served from one L2.
#include <vector>

#include "kernels.hpp"
#include "sdsp_runtime.hpp"

namespace sdsp {

// one complex value: two scalar registers; 8-byte aligned so LDS moves are ds_*_b64
struct __attribute__((aligned(8))) c2 {
    float x, y;
};

__device__ __forceinline__ c2 ld_c2(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(c2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
// buffer resource over [p, p+bytes) for a wave-uniform pointer
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, bytes, 0x00020000);
}

// the spec's complex product: (fma(w.re, z.re, -(w.im z.im)), fma(w.re, z.im, w.im z.re))
__device__ __forceinline__ c2 cmulf(c2 w, c2 z) {
    return {__builtin_fmaf(w.x, z.x, -(w.y * z.y)), __builtin_fmaf(w.x, z.y, w.y * z.x)};
}

// radix-4 butterfly of sdsp_fft_spec.h; TW = false: p = 0, no products
template <bool TW>
__device__ __forceinline__ void bfly4(c2 a, c2 b, c2 c, c2 d, c2 w1, c2 w2, c2 w3, c2& y0, c2& y1, c2& y2, c2& y3) {
    const c2 apc = {a.x + c.x, a.y + c.y}, amc = {a.x - c.x, a.y - c.y};
    const c2 bpd = {b.x + d.x, b.y + d.y}, bmd = {b.x - d.x, b.y - d.y};
    const c2 t1 = {amc.x + bmd.y, amc.y - bmd.x};  // amc + (-i)(b - d)
    const c2 t2 = {apc.x - bpd.x, apc.y - bpd.y};
    const c2 t3 = {amc.x - bmd.y, amc.y + bmd.x};  // amc - (-i)(b - d)
    y0 = {apc.x + bpd.x, apc.y + bpd.y};
    if constexpr (TW) {
        y1 = cmulf(w1, t1);
        y2 = cmulf(w2, t2);
        y3 = cmulf(w3, t3);
    } else {
        y1 = t1;
        y2 = t2;
        y3 = t3;
    }
}

// 16 LDS elements p[ST k], k < 16, read as 16 single ds_read_b64 (the compiler pairs such reads
// into ds_read2_b64, 8 LDS cycles per pair against 2 per single read, MI355X_MICROARCH.md LDS
// table; a volatile access does not stop it), then waited for
template <int ST>
__device__ __forceinline__ void lds_ld16(const c2* p, c2 v[16]) {
    typedef __attribute__((address_space(3))) const c2 lds_c2;
    const uint32_t a = (uint32_t)(uintptr_t)(lds_c2*)p;
    uint64_t r[16];
    asm volatile(
        "ds_read_b64 %0, %16 offset:%17\n ds_read_b64 %1, %16 offset:%18\n ds_read_b64 %2, %16 offset:%19\n"
        "ds_read_b64 %3, %16 offset:%20\n ds_read_b64 %4, %16 offset:%21\n ds_read_b64 %5, %16 offset:%22\n"
        "ds_read_b64 %6, %16 offset:%23\n ds_read_b64 %7, %16 offset:%24\n ds_read_b64 %8, %16 offset:%25\n"
        "ds_read_b64 %9, %16 offset:%26\n ds_read_b64 %10, %16 offset:%27\n ds_read_b64 %11, %16 offset:%28\n"
        "ds_read_b64 %12, %16 offset:%29\n ds_read_b64 %13, %16 offset:%30\n ds_read_b64 %14, %16 offset:%31\n"
        "ds_read_b64 %15, %16 offset:%32\n s_waitcnt lgkmcnt(0)"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]),
          "=&v"(r[8]), "=&v"(r[9]), "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]), "=&v"(r[15])
        : "v"(a), "n"(0), "n"(8 * ST), "n"(16 * ST), "n"(24 * ST), "n"(32 * ST), "n"(40 * ST), "n"(48 * ST), "n"(56 * ST),
          "n"(64 * ST), "n"(72 * ST), "n"(80 * ST), "n"(88 * ST), "n"(96 * ST), "n"(104 * ST), "n"(112 * ST), "n"(120 * ST)
        : "memory");
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = __builtin_bit_cast(c2, r[k]);
}

__device__ __forceinline__ int lpad(int i) { return i + (i >> 4); }
#define P17 17
#define P272 272
#define PADSHIFT 1

// Barrier over the threads of one frame: a frame of TPF = 64 threads is one wave, whose LDS
// operations complete in order, so a wave-scope fence + wave barrier replaces the workgroup
// barrier and the frames of a workgroup run independently.
template <int TPF>
__device__ __forceinline__ void frame_sync() {
    if constexpr (TPF == 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

// Correctly rounded f32 sqrt.  For x in [2^-96, inf) this is exactly the sequence hipcc emits
// for sqrtf under -fhip-fp32-correctly-rounded-divide-sqrt (v_sqrt_f32, then the +-1 ulp
// FMA-residual correction) without its small-input rescaling and special-value select; other
// inputs (0, tiny, inf, NaN) take the compiler's full sqrtf.  tools/check_sqrt.hip: identical
// to sqrtf on every non-negative f32.
__device__ __forceinline__ float sqrt_cr(float x) {
    if (__builtin_expect(x >= 0x1p-96f && x < __builtin_huge_valf(), 1)) {
        float s = __builtin_amdgcn_sqrtf(x);
        const float sm = __uint_as_float(__float_as_uint(s) - 1u);
        const float sp = __uint_as_float(__float_as_uint(s) + 1u);
        const float rm = __builtin_fmaf(-sm, s, x);
        const float rp = __builtin_fmaf(-sp, s, x);
        s = rm <= 0.0f ? sm : s;
        s = rp > 0.0f ? sp : s;
        return s;
    }
    return __builtin_sqrtf(x);
}

// Correctly rounded f32 sqrt without compare masks or branches, for x = +0 and x in [2^-96, inf):
// Markstein's step from the hardware reciprocal square root, y ~ 1/sqrt(x): s0 = x y, h = y / 2,
// r = x - s0^2 (exact by FMA), s = s0 + r h.  x = +0 takes y from max(x, 2^-126), which is finite,
// so s0 = +0 and s = +0.  tools/check_sqrt2.hip checks it against the correctly rounded sqrtf on
// every such f32 on gfx950 (the only mismatch is x = +inf).  5 VALU + 1 transcendental, against 11
// + 1 for the +-1 ulp residual correction of v_sqrt's result it replaces.  Inputs outside that set
// (subnormal-scale x, inf, NaN) are recorded in lo / hi (min of bits - 1, max of bits) for the
// caller's fix-up pass.
__device__ __forceinline__ float sqrt_fast(float x, uint32_t& lo, uint32_t& hi) {
    const uint32_t u = __float_as_uint(x);
    lo = min(lo, u - 1u);
    hi = max(hi, u);
    const float y = __builtin_amdgcn_rsqf(__builtin_fmaxf(x, 0x1p-126f));
    const float s0 = x * y, h = 0.5f * y;
    return __builtin_fmaf(__builtin_fmaf(-s0, s0, x), h, s0);
}
// true when some input of sqrt_fast was outside its exact range
__device__ __forceinline__ bool sqrt_fast_missed(uint32_t lo, uint32_t hi) {
    return lo < 0x0F7FFFFFu || hi >= 0x7F800000u;  // (0, 2^-96) or inf / NaN
}

// Two radix-4 stages, (n, s) then (n/4, 4s), on v[j' + 4j] = x[q + s(p' + (n/16)(j' + 4j))].
// On return v[jA + 4jB] = z[q + 16 s p' + s(jA + 4jB)].  w[0..11] = stage-A twiddles
// W^{jA (p' + j' n/16) M/n} at index 3 j' + jA - 1, w[12..14] = stage-B W^{jB p' 4M/n}.
// LAST (p' = 0 for every lane, the last pass): stage A's j' = 0 butterfly and all of stage B
// have p = 0, so they carry no products.
template <bool LAST>
__device__ __forceinline__ void radix16(c2 v[16], const c2 w[15]) {
    c2 u[16];
#pragma unroll
    for (int jp = 0; jp < 4; jp++) {
        if (LAST && jp == 0)
            bfly4<false>(v[0], v[4], v[8], v[12], w[0], w[0], w[0], u[0], u[1], u[2], u[3]);
        else
            bfly4<true>(v[jp], v[jp + 4], v[jp + 8], v[jp + 12], w[3 * jp + 0], w[3 * jp + 1], w[3 * jp + 2],
                        u[jp * 4 + 0], u[jp * 4 + 1], u[jp * 4 + 2], u[jp * 4 + 3]);
    }
#pragma unroll
    for (int ja = 0; ja < 4; ja++)
        bfly4<!LAST>(u[0 * 4 + ja], u[1 * 4 + ja], u[2 * 4 + ja], u[3 * 4 + ja], w[12], w[13], w[14], v[ja + 0],
                     v[ja + 4], v[ja + 8], v[ja + 12]);
}

// radix16 whose 15 twiddles come from a loader (tw(j) = w[j] of radix16) fetched per butterfly:
// stage A's butterfly j' takes tw(3 j' .. 3 j' + 2) just before it runs and stage B's three are
// fetched after stage A, so at most 3 twiddles are live instead of 15 (k_stft_slide8w3's pass 2,
// whose LDS twiddles otherwise need 30 VGPRs beside the register ring at the 168-VGPR limit)
template <typename TW>
__device__ __forceinline__ void radix16_tw(c2 v[16], TW tw) {
    c2 u[16];
#pragma unroll
    for (int jp = 0; jp < 4; jp++) {
        const c2 w1 = tw(3 * jp + 0), w2 = tw(3 * jp + 1), w3 = tw(3 * jp + 2);
        bfly4<true>(v[jp], v[jp + 4], v[jp + 8], v[jp + 12], w1, w2, w3, u[jp * 4 + 0], u[jp * 4 + 1],
                    u[jp * 4 + 2], u[jp * 4 + 3]);
    }
    const c2 b1 = tw(12), b2 = tw(13), b3 = tw(14);
#pragma unroll
    for (int ja = 0; ja < 4; ja++)
        bfly4<true>(u[0 * 4 + ja], u[1 * 4 + ja], u[2 * 4 + ja], u[3 * 4 + ja], b1, b2, b3, v[ja + 0], v[ja + 4],
                    v[ja + 8], v[ja + 12]);
}

template <int M>
struct StftShape {
    static constexpr int TPF = M / 16;                                   // threads per frame
    static constexpr int NPASS = (M == 4096) ? 3 : (M == 1024) ? 2 : 0;  // radix-16 passes
    static constexpr int NPAIR = (M / 2 + TPF - 1) / TPF;               // post pairs per thread
    static constexpr int RT_SPECIAL = NPAIR * 2 * TPF;                  // rt[0], rt[M], rt[M/2], tw[0]
};

// one frame of k_stft_mag (frame group = the threads with the same threadIdx.x / TPF)
template <int NFFT, bool FRAME_MAX>
__device__ __forceinline__ void stft_mag_frame(const float* __restrict__ samples, const uint64_t* __restrict__ frame_pfx,
                                               int n_tracks, uint64_t gg, bool live, const uint64_t* __restrict__ src_off,
                                               const float* __restrict__ gain, int hop, const float* __restrict__ window,
                                               const cx* __restrict__ twp, const cx* __restrict__ rtp,
                                               float* __restrict__ mags, const uint64_t* __restrict__ mag_row0,
                                               int stride, float* __restrict__ frame_max) {
    constexpr int M = NFFT / 2;
    using S = StftShape<M>;
    constexpr int TPF = S::TPF;
    constexpr int FPB = 256 / TPF;    // frames per workgroup
    constexpr int PADM = M + PADSHIFT * M / 16;  // padded LDS slots per frame
    static_assert(S::NPASS > 0, "supported sizes: N = 2048, 8192");
    __shared__ c2 lds[FPB * PADM];
    __shared__ float red[4];

    const int lt = threadIdx.x % TPF;  // thread within frame
    const int fl = threadIdx.x / TPF;  // frame within workgroup
    const int trk = find_track(frame_pfx, n_tracks, gg);
    const uint64_t f = gg - frame_pfx[trk];
    const float gn = gain[trk];
    c2* buf = lds + fl * PADM;
    const __amdgpu_buffer_rsrc_t rx = rsrc_of(samples + src_off[trk] + f * (uint64_t)hop, 4u * NFFT);
    const __amdgpu_buffer_rsrc_t rw = rsrc_of(window, 4u * NFFT);
    const __amdgpu_buffer_rsrc_t rtw = rsrc_of(twp, 8u * 15u * (TPF + TPF / 16 + 1));
    const __amdgpu_buffer_rsrc_t rrt = rsrc_of(rtp, 8u * (S::RT_SPECIAL + 4));
    const int vo = 8 * lt;  // every table below is [item][lane] with 8-byte entries

    // The overflow rule of the STFT section (sdsp_fft_spec.h): the frame is evaluated with the
    // window's 2^32 (pre = 1, |X| = 2^-33 sqrt(.)); if some |Y|^2 overflowed to +inf, the whole
    // frame is evaluated again with the windowed samples times 2^-33 (Y = X, the reference's own
    // range, src/features/chroma/extractor.rs:352) and |X| = sqrt(.).
    float pre = 1.0f, post = 0x1p-33f, mx = 0.0f;
    for (int attempt = 0; attempt < 2; attempt++) {
        bool ovf = false;
        c2 v[16], w[15];
        // pass 1 (n = M, s = 1, p' = lt): z[idx] = (x[2idx], x[2idx+1]) * gain * window, idx = lt + TPF k
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const c2 xs = ld_c2(rx, vo, 8 * TPF * k);
            const c2 ws = ld_c2(rw, vo, 8 * TPF * k);
            v[k] = {((xs.x * gn) * ws.x) * pre, ((xs.y * gn) * ws.y) * pre};
        }
#pragma unroll
        for (int j = 0; j < 15; j++)
            w[j] = ld_c2(rtw, vo, 8 * TPF * j);
        radix16<false>(v, w);
        {
            const int b0 = P17 * lt;  // lpad(16 lt + k) = 17 lt + k
#pragma unroll
            for (int k = 0; k < 16; k++) buf[b0 + k] = v[k];
        }
        frame_sync<TPF>();
        // further radix-16 passes: (n, s) = (M/16, 16), (M/256, 256)
#pragma unroll
        for (int pass = 1; pass < S::NPASS; pass++) {
            const int s = pass == 1 ? 16 : 256;
            const int m1 = (pass == 1 ? M / 16 : M / 256) / 16;  // n / 16
            const int q = lt % s, pp = pass == 2 ? 0 : lt / s;  // lt < TPF = 256 = s on pass 2
            // reads x[q + s pp + s m1 k]; s m1 is a multiple of 16, so lpad = lpad(q + s pp) + (17/16) s m1 k
            const int rb = lpad(q + s * pp), rs = s * m1 + PADSHIFT * (s * m1) / 16;
#pragma unroll
            for (int j = 0; j < 15; j++) {
                // pass 1: one entry per p' (TPF/16 of them, shared by 16 lanes); pass 2: p' = 0 for
                // every lane, so the 15 twiddles are wave-uniform scalar loads
                if (pass == 1) {
                    w[j] = ld_c2(rtw, 8 * pp, 8 * (15 * TPF + j * (TPF / 16)));
                } else {
                    const cx t = twp[15 * TPF + 15 * (TPF / 16) + j];
                    w[j] = c2{t.re, t.im};
                }
            }
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = buf[rb + rs * k];
            frame_sync<TPF>();
            if (pass == 2)
                radix16<true>(v, w);
            else
                radix16<false>(v, w);
            // writes z[q + 16 s pp + s k]:  s = 16 -> (q + 272 pp) + 17 k;  s = 256 (pp = 0) -> lpad(q) + 272 k
            if (s == 16) {
                const int wb = q + P272 * pp;
#pragma unroll
                for (int k = 0; k < 16; k++) buf[wb + P17 * k] = v[k];
            } else {  // s = 256 only for M = 4096 (m1 = 1): z[q + 256 k], lpad = lpad(q) + 272 k
#pragma unroll
                for (int k = 0; k < 16; k++) buf[rb + P272 * k] = v[k];
            }
            frame_sync<TPF>();
        }
        // trailing radix-4 stage (M = 16^2 * 4): n = 4, s = M/4, p = 0 (no products)
        if constexpr (M == 1024) {
            constexpr int s = M / 4;
#pragma unroll
            for (int r = 0; r < s / TPF; r++) {
                const int q = lt + TPF * r;
                const int b = lpad(q);  // lpad(q + j s) = b + 272 j (s = 256)
                c2 y0, y1, y2, y3;
                bfly4<false>(buf[b], buf[b + P272], buf[b + 2 * P272], buf[b + 3 * P272], c2{}, c2{}, c2{}, y0, y1, y2, y3);
                buf[b] = y0;
                buf[b + P272] = y1;
                buf[b + 2 * P272] = y2;
                buf[b + 3 * P272] = y3;
            }
            frame_sync<TPF>();
        }
        // real-FFT post-processing, |X[k]|, k = 0..M (sdsp_fft_spec.h, STFT section):
        //   S = Z[k] + conj(Z[M-k]),  D = Z[k] - conj(Z[M-k]),  D' = (D.im, -D.re),
        //   Y = S + rt[k] D' in FMA form,  |X[k]| = 0.5 * sqrt(fma(Y.re, Y.re, Y.im * Y.im)).
        // Bins k and M-k read the same pair (Z[k], Z[M-k]); the partner's S and D' are the
        // conjugates of this bin's (exactly, up to the sign of zero, which |X| cannot see), so each
        // pair is read and combined once.
        float* out = mags + (mag_row0[trk] + f) * (uint64_t)stride;
        mx = 0.0f;
        auto mag_of = [&](float sx, float sy, float dx, float dy, c2 wt) {  // S = (sx, sy), D' = (dx, dy)
            const float yx = __builtin_fmaf(wt.x, dx, __builtin_fmaf(-wt.y, dy, sx));
            const float yy = __builtin_fmaf(wt.x, dy, __builtin_fmaf(wt.y, dx, sy));
            const float e = __builtin_fmaf(yx, yx, yy * yy);
            ovf |= e == __builtin_huge_valf();
            return post * sqrt_cr(e);
        };
        auto put = [&](int k, float mag) {
            if (live) out[k] = mag;
            if (FRAME_MAX) mx = sd_maxf(mx, mag);
        };
        struct SD {
            float sx, sy, dx, dy;
        };
        auto pair_sd = [&](int ik, int ir) {  // LDS indices of Z[k], Z[M-k]
            const c2 Zk = buf[ik];
            const c2 Zr = buf[ir];
            // S = Zk + conj(Zr);  D = Zk - conj(Zr);  D' = (D.im, -D.re)
            return SD{Zk.x + Zr.x, Zk.y - Zr.y, Zk.y + Zr.y, -(Zk.x - Zr.x)};
        };
        c2 wk[S::NPAIR], wm[S::NPAIR];
#pragma unroll
        for (int j = 0; j < S::NPAIR; j++) {
            wk[j] = ld_c2(rrt, vo, 8 * TPF * (2 * j));
            wm[j] = ld_c2(rrt, vo, 8 * TPF * (2 * j + 1));
        }
#pragma unroll
        for (int j = 0; j < S::NPAIR; j++) {
            const int k = 1 + lt + TPF * j;  // k < M/2 except possibly on the last j
            if (j + 1 < S::NPAIR || k < M / 2) {
                const SD a = pair_sd(lpad(k), lpad(M - k));
                put(k, mag_of(a.sx, a.sy, a.dx, a.dy, wk[j]));
                put(M - k, mag_of(a.sx, -a.sy, a.dx, -a.dy, wm[j]));
            }
        }
        if (lt == 0) {  // k = 0 and k = M both read (Z[0], Z[0]); k = M/2 reads (Z[M/2], Z[M/2])
            const SD a = pair_sd(0, 0);
            put(0, mag_of(a.sx, a.sy, a.dx, a.dy, ld_c2(rrt, 0, 8 * S::RT_SPECIAL)));
            put(M, mag_of(a.sx, a.sy, a.dx, a.dy, ld_c2(rrt, 0, 8 * (S::RT_SPECIAL + 1))));
        } else if (lt == 1) {
            const SD a = pair_sd(lpad(M / 2), lpad(M / 2));
            put(M / 2, mag_of(a.sx, a.sy, a.dx, a.dy, ld_c2(rrt, 0, 8 * (S::RT_SPECIAL + 2))));
        }
        const bool any = TPF == 64 ? __builtin_amdgcn_ballot_w64(ovf) != 0 : __syncthreads_or(ovf) != 0;
        if (!any) break;
        frame_sync<TPF>();  // this attempt's LDS reads are done before the next one's writes
        pre = 0x1p-33f;
        post = 1.0f;
    }
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

// k_stft_mag: one frame per frame group (the general kernel: any hop).  With `redo` (the sliding
// kernel's list: redo[0] = count, then global frame indices) it recomputes only the listed frames,
// grid-striding over the list.
template <int NFFT, bool FRAME_MAX>
__global__ __launch_bounds__(256) void k_stft_mag(const float* __restrict__ samples,
                                                  const uint64_t* __restrict__ frame_pfx, int n_tracks,
                                                  uint64_t total_frames, const uint64_t* __restrict__ src_off,
                                                  const float* __restrict__ gain, int hop,
                                                  const float* __restrict__ window, const cx* __restrict__ twp,
                                                  const cx* __restrict__ rtp, float* __restrict__ mags,
                                                  const uint64_t* __restrict__ mag_row0, int stride,
                                                  float* __restrict__ frame_max, const uint32_t* __restrict__ redo) {
    if (redo) {
        constexpr int FPB = 256 / StftShape<NFFT / 2>::TPF;
        const uint32_t n = redo[0];
        for (uint32_t e = blockIdx.x * FPB + threadIdx.x / StftShape<NFFT / 2>::TPF; e < n; e += gridDim.x * FPB)
            stft_mag_frame<NFFT, FRAME_MAX>(samples, frame_pfx, n_tracks, (uint64_t)redo[1 + e], true, src_off, gain,
                                            hop, window, twp, rtp, mags, mag_row0, stride, frame_max);
        return;
    }
    const uint64_t g = (uint64_t)xcd_block(blockIdx.x, gridDim.x) * (256 / StftShape<NFFT / 2>::TPF) +
                       threadIdx.x / StftShape<NFFT / 2>::TPF;
    const bool live = g < total_frames;
    stft_mag_frame<NFFT, FRAME_MAX>(samples, frame_pfx, n_tracks, live ? g : total_frames - 1, live, src_off, gain,
                                    hop, window, twp, rtp, mags, mag_row0, stride, frame_max);
}

// ---------------------------------------------------------------------------------------------
// k_stft_gen: the STFT of any power-of-two frame size N in [STFT_GEN_MIN, STFT_GEN_MAX] other
// than the tuned 2048 / 8192 (AnalysisConfig::frame_size is a free knob, src/config.rs).  The
// spec's algorithm stage by stage: one 256-thread workgroup per frame, z = M = N/2 complex values
// ping-ponged between two LDS buffers (dynamic LDS, 8 N bytes), radix-4 stages then the radix-2
// stage when log2 M is odd, the real-FFT post-processing bin by bin with the symmetric post
// twiddles, |X| by the correctly rounded sqrt.  tw / rt are the spec's plain tables.  Each
// butterfly and each bin evaluates exactly the expressions of oracle/o_fft.cpp stft_fft_complex /
// stft_mag, so the magnitudes are bit-identical to the tuned kernels' (same spec).
template <bool FRAME_MAX>
__global__ __launch_bounds__(256) void k_stft_gen(int N, const float* __restrict__ samples,
                                                  const uint64_t* __restrict__ frame_pfx, int n_tracks,
                                                  uint64_t total_frames, const uint64_t* __restrict__ src_off,
                                                  const float* __restrict__ gain, int hop,
                                                  const float* __restrict__ window, const cx* __restrict__ tw,
                                                  const cx* __restrict__ rt, float* __restrict__ mags,
                                                  const uint64_t* __restrict__ mag_row0, int stride,
                                                  float* __restrict__ frame_max) {
    extern __shared__ c2 gen_lds[];
    __shared__ float red[4];
    const uint64_t g = xcd_block(blockIdx.x, gridDim.x);
    if (g >= total_frames) return;  // whole workgroup: uniform
    const int M = N >> 1, lgm = 31 - __builtin_clz((unsigned)M);
    const int trk = find_track(frame_pfx, n_tracks, g);
    const uint64_t f = g - frame_pfx[trk];
    const float gn = gain[trk];
    const float* x = samples + src_off[trk] + f * (uint64_t)hop;
    // the STFT section's overflow rule (see stft_mag_frame)
    float pre = 1.0f, post = 0x1p-33f, mx = 0.0f;
    for (int attempt = 0; attempt < 2; attempt++) {
        bool ovf = false;
        c2* a = gen_lds;
        c2* b = gen_lds + M;
        for (int j = threadIdx.x; j < M; j += 256)
            a[j] = c2{((x[2 * j] * gn) * window[2 * j]) * pre, ((x[2 * j + 1] * gn) * window[2 * j + 1]) * pre};
        __syncthreads();
        // radix-4 stages: (n, s) = (M, 1), (M/4, 4), ...; butterfly u = p s + q
        int lgs = 0;
        for (int lgn = lgm; lgn >= 2; lgn -= 2, lgs += 2) {
            const int s = 1 << lgs, m = 1 << (lgn - 2), tstep = M >> lgn;
            for (int u = threadIdx.x; u < (M >> 2); u += 256) {
                const int q = u & (s - 1), p = u >> lgs;
                c2 y0, y1, y2, y3;
                const c2 va = a[q + s * p], vb = a[q + s * (p + m)], vc = a[q + s * (p + 2 * m)],
                         vd = a[q + s * (p + 3 * m)];
                if (p) {
                    const cx w1 = tw[p * tstep], w2 = tw[2 * p * tstep], w3 = tw[3 * p * tstep];
                    bfly4<true>(va, vb, vc, vd, c2{w1.re, w1.im}, c2{w2.re, w2.im}, c2{w3.re, w3.im}, y0, y1, y2, y3);
                } else {
                    bfly4<false>(va, vb, vc, vd, c2{}, c2{}, c2{}, y0, y1, y2, y3);
                }
                const int o = q + s * 4 * p;
                b[o] = y0;
                b[o + s] = y1;
                b[o + 2 * s] = y2;
                b[o + 3 * s] = y3;
            }
            __syncthreads();
            c2* t = a;
            a = b;
            b = t;
        }
        if (lgm & 1) {  // radix-2 stage: s = M/2
            const int s = M >> 1;
            for (int q = threadIdx.x; q < s; q += 256) {
                const c2 va = a[q], vb = a[q + s];
                b[q] = c2{va.x + vb.x, va.y + vb.y};
                b[q + s] = c2{va.x - vb.x, va.y - vb.y};
            }
            __syncthreads();
            a = b;
        }
        // post-processing, k = 0..M (oracle/o_fft.cpp stft_mag)
        float* out = mags + (mag_row0[trk] + f) * (uint64_t)stride;
        mx = 0.0f;
        for (int k = threadIdx.x; k <= M; k += 256) {
            const c2 zk = a[k & (M - 1)], zr = a[(M - k) & (M - 1)];
            const cx r = rt[k > (M >> 1) ? M - k : k];
            const c2 w = k > (M >> 1) ? c2{-r.re, r.im} : c2{r.re, r.im};
            const float sre = zk.x + zr.x, sim = zk.y - zr.y;
            const float dre = zk.y + zr.y, dim = -(zk.x - zr.x);
            const float yre = __builtin_fmaf(w.x, dre, __builtin_fmaf(-w.y, dim, sre));
            const float yim = __builtin_fmaf(w.x, dim, __builtin_fmaf(w.y, dre, sim));
            const float e = __builtin_fmaf(yre, yre, yim * yim);
            ovf |= e == __builtin_huge_valf();
            const float mag = post * sqrt_cr(e);
            out[k] = mag;
            if (FRAME_MAX) mx = sd_maxf(mx, mag);
        }
        if (!__syncthreads_or(ovf)) break;
        pre = 0x1p-33f;
        post = 1.0f;
    }
    if (FRAME_MAX) {
        mx = wave_max(mx);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            float m = red[0];
            for (int i = 1; i < 4; i++) m = sd_maxf(m, red[i]);
            frame_max[mag_row0[trk] + f] = m;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Sliding-strip STFT (the pipeline's kernel for hops that are a multiple of 2*TPF complex
// values: 8192/512, 8192/1024, 2048/256, 2048/512, 2048/1024).  Same arithmetic as k_stft_mag,
// different data movement, because the isolated profile of k_stft_mag showed it bound by what it
// re-reads per frame, not by its arithmetic (window + twiddle tables ~100 KB and
// the 16x-overlapped samples 32 KB per 8192-point frame, all from L2):
//  * a strip = up to STRIP_T consecutive frames of one track, processed in order by one
//    frame-group (8192: the 256-thread workgroup; 2048: one wave);
//  * window, pass-1 and pass-2 twiddles and post twiddles are loaded into registers once per strip;
//  * thread lt holds z[lt + TPF k], k = 0..15, of the current frame in a register ring.  The
//    next frame starts hop/2 = S*TPF complex values later, so its element k is the current
//    element k + S: the ring shifts by S and only S new values per thread are loaded (prefetched
//    one frame ahead);
//  * two LDS buffers: pass 1 writes A, pass 2 reads A and writes B, the last pass reads B into
//    registers.  Its columns are assigned so that each real-FFT pair (k, M-k) meets in one thread
//    (N = 2048) or in lanes l and l^32 of one wave, exchanged by ds_bpermute (N = 8192), so the
//    post-processing runs from registers: two barriers per frame, no barrier between a pass's
//    reads and its writes, and two LDS round trips instead of three;
//  * the STFT post twiddles are the spec's symmetric ones, rt[M-k] = (-rt[k].re, rt[k].im), so
//    bin M-k needs no table entry of its own;
//  * the correctly rounded sqrt is sqrt_fast; a frame where it met an input outside its exact
//    range (magnitudes of subnormal scale, inf, NaN) is appended to a redo list that k_stft_mag
//    recomputes right after (launch_stft).
constexpr int STRIP_T = 64;

// Last-pass columns of the sliding kernel, chosen so that the real-FFT pairs (k, M-k) meet in
// registers.  Column c holds Z[c + 256 m]; its pairs lie in column 256 - c (mod 256).
//  N = 8192 (16 per column, 256 threads): lanes l and l + 32 of a wave hold partner columns
//    c = 32 w + l and 256 - c; wave 0's lanes 0 / 32 hold the self-paired columns 0 / 128.
//  N = 2048 (4 per column, one wave): thread t holds columns (t, 256 - t) and (128 - t, 128 + t);
//    thread 0 holds (0, 128) and (64, 192).
__host__ __device__ inline int slide_col8(int lt) {
    const int w = lt >> 6, l = lt & 63, base = 32 * w + (l & 31);
    return l < 32 ? base : (base == 0 ? 128 : 256 - base);
}
__host__ __device__ inline void slide_cols2(int t, int* a, int* a2, int* b, int* b2) {
    *a = t;
    *a2 = t ? 256 - t : 128;
    *b = t ? 128 - t : 64;
    *b2 = t ? 128 + t : 192;
}
// The bin of each post slot (own bin k; the partner bin is M - k) of thread lt, slot j < 8.
//  N = 8192: k = col + 256 j.  N = 2048: slots 0-3 pair (a, a2), 4-7 pair (b, b2), k = col + 256 j';
//  thread 0's first four slots are {0, 256, 128, 384} (columns 0 and 128 pair within themselves).
__host__ __device__ inline int slide_bin(int M, int lt, int j) {
    if (M == 4096) return slide_col8(lt) + 256 * j;
    int a, a2, b, b2;
    slide_cols2(lt, &a, &a2, &b, &b2);
    if (j >= 4) return b + 256 * (j - 4);
    if (lt == 0) {
        const int t0[4] = {0, 256, 128, 384};
        return t0[j];
    }
    return a + 256 * j;
}
// rtp offset of the sliding kernel's post table: [slot j][lane] rt(slide_bin), then rt(M/2)
template <int M>
constexpr int slide_rt_base() {
    return StftShape<M>::RT_SPECIAL + 4;
}

template <int NFFT, int S, bool FRAME_MAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_stft_slide(
    const float* __restrict__ samples, const uint64_t* __restrict__ frame_pfx, const uint64_t* __restrict__ strip_pfx,
    int n_tracks, uint64_t n_strips, const uint64_t* __restrict__ src_off, const float* __restrict__ gain, int hop,
    const float* __restrict__ window, const cx* __restrict__ twp, const cx* __restrict__ rtp, float* __restrict__ mags,
    const uint64_t* __restrict__ mag_row0, int stride, float* __restrict__ frame_max, uint32_t* __restrict__ redo) {
    constexpr int M = NFFT / 2;
    using SH = StftShape<M>;
    constexpr int TPF = SH::TPF;
    constexpr int FPB = 256 / TPF;               // frame groups (strips) per workgroup
    constexpr int PADM = M + PADSHIFT * M / 16;  // padded LDS slots per frame buffer
    static_assert(SH::NPASS > 0 && S >= 1 && S <= 16, "supported: N = 2048, 8192; hop = S * 2 * TPF");
    __shared__ c2 lds[FPB * 2 * PADM];
    __shared__ uint32_t miss_flag[2];  // N = 8192: frame i's "some wave missed" flag at [i & 1]

    const int lt = threadIdx.x % TPF;
    const int fl = threadIdx.x / TPF;
    // wave-uniform by construction (a frame group is whole waves); readfirstlane lets the compiler
    // keep the strip's scalars and buffer descriptors in SGPRs
    const uint64_t strip =
        (uint64_t)__builtin_amdgcn_readfirstlane((int)((uint64_t)xcd_block(blockIdx.x, gridDim.x) * FPB + fl));
    if (strip >= n_strips) return;  // only whole frame groups: a wave (TPF = 64) or the workgroup (FPB = 1)
    if (TPF == 256 && threadIdx.x < 2) miss_flag[threadIdx.x] = 0;  // ordered by frame 0's barriers
    const int trk = find_track(strip_pfx, n_tracks, strip);
    const uint64_t F = frame_pfx[trk + 1] - frame_pfx[trk];
    const uint64_t f0 = (strip - strip_pfx[trk]) * (uint64_t)STRIP_T;
    const int nf = (int)(F - f0 < (uint64_t)STRIP_T ? F - f0 : (uint64_t)STRIP_T);
    const float gn = gain[trk];
    c2* bufA = lds + fl * 2 * PADM;
    c2* bufB = bufA + PADM;
    const int vo = 8 * lt;
    // the strip's samples: frame f0 + i starts at complex index (f0 + i) * hop / 2
    const uint64_t cstart = f0 * (uint64_t)(hop / 2);
    const uint64_t clen = (uint64_t)(nf - 1) * (uint64_t)(hop / 2) + (uint64_t)M;  // complex values the strip reads
    const float* sbase = samples + src_off[trk] + 2 * cstart;
    const __amdgpu_buffer_rsrc_t rx = rsrc_of(sbase, (uint32_t)(8u * clen));
    const __amdgpu_buffer_rsrc_t rw = rsrc_of(window, 4u * NFFT);
    const __amdgpu_buffer_rsrc_t rtw = rsrc_of(twp, 8u * 15u * (TPF + TPF / 16 + 1));
    const __amdgpu_buffer_rsrc_t rrt = rsrc_of(rtp, 8u * (slide_rt_base<M>() + 8 * TPF + 1));

    // per-strip constants
    c2 win[16], tw1[15], tw2[15], wk[8];
    c2 ring[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {  // the ring holds x * gain (the normalised samples, src/lib.rs:124)
        const c2 x = ld_c2(rx, vo, 8 * TPF * k);
        ring[k] = {x.x * gn, x.y * gn};
    }
#pragma unroll
    for (int k = 0; k < 16; k++) win[k] = ld_c2(rw, vo, 8 * TPF * k);
#pragma unroll
    for (int j = 0; j < 15; j++) tw1[j] = ld_c2(rtw, vo, 8 * TPF * j);
    const int pp2 = lt / 16;  // pass 2 (s = 16): p' = lt / 16
#pragma unroll
    for (int j = 0; j < 15; j++) tw2[j] = ld_c2(rtw, 8 * pp2, 8 * (15 * TPF + j * (TPF / 16)));
#pragma unroll
    for (int j = 0; j < 8; j++) wk[j] = ld_c2(rrt, vo, 8 * (slide_rt_base<M>() + TPF * j));
    c2 tw3[15];  // pass 3 (M = 4096): p' = 0, wave-uniform
    if constexpr (M == 4096) {
#pragma unroll
        for (int j = 0; j < 15; j++) {
            const cx t = twp[15 * TPF + 15 * (TPF / 16) + j];
            tw3[j] = c2{t.re, t.im};
        }
    }
    const c2 rtH = ld_c2(rrt, 0, 8 * (slide_rt_base<M>() + 8 * TPF));  // bin M/2
    // last-pass columns and the bins of the post slots
    int colA, colA2, colB, colB2;
    if constexpr (M == 4096) {
        colA = slide_col8(lt);
        colA2 = colB = colB2 = 0;
    } else {
        slide_cols2(lt, &colA, &colA2, &colB, &colB2);
    }
    const bool self0 = M == 4096 ? (threadIdx.x == 0) : (lt == 0);  // the column-0 thread
    const bool self128 = M == 4096 && threadIdx.x == 32;             // the column-128 lane (N = 8192)
    // N = 8192: the partner lane (l ^ 32), or the lane itself for the self-paired columns
    const int src_lane = (self0 || self128) ? (threadIdx.x & 63) : ((threadIdx.x & 63) ^ 32);

    // every per-strip load has landed before the frame loop: the loop header then carries no
    // pending load, so the compiler does not wait there for the previous frame's stores
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    for (int i = 0; i < nf; i++) {
        const uint64_t f = f0 + (uint64_t)i;
        // prefetch the next frame's S new ring values: z[(i+1) h + lt + TPF (16 - S + s)].  After
        // the strip's last frame the offsets are past the descriptor's range, where buffer loads
        // return 0 without touching memory, so the load needs no branch (a conditional load
        // makes the compiler wait for it at once).
        c2 nxt[S];
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) nxt[s2] = ld_c2(rx, vo, 8 * ((i + 1) * (hop / 2) + TPF * (16 - S + s2)));
        c2 v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = {ring[k].x * win[k].x, ring[k].y * win[k].y};
        // pass 1 (n = M, s = 1, p' = lt) -> A
        radix16<false>(v, tw1);
#pragma unroll
        for (int k = 0; k < 16; k++) bufA[P17 * lt + k] = v[k];
        frame_sync<TPF>();
        if constexpr (TPF == 256) {
            // frame i - 1's flag is final (its waves set it before this barrier); cleared before
            // this frame's second barrier, so before frame i + 1 can set it again
            if (threadIdx.x == 0 && i > 0 && miss_flag[(i - 1) & 1]) {
                miss_flag[(i - 1) & 1] = 0;
                redo[1 + atomicAdd(redo, 1u)] = (uint32_t)(frame_pfx[trk] + f - 1);
            }
        }
        // pass 2 (n = M/16, s = 16): A -> B
        {
            constexpr int s2 = 16, m1 = (M / 16) / 16;
            const int q = lt % s2;
            const int rb = lpad(q + s2 * pp2), rs = s2 * m1 + PADSHIFT * (s2 * m1) / 16;
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = bufA[rb + rs * k];
            radix16<false>(v, tw2);
            const int wb = q + P272 * pp2;
#pragma unroll
            for (int k = 0; k < 16; k++) bufB[wb + P17 * k] = v[k];
        }
        frame_sync<TPF>();
        // last pass, then the post-processing from registers (sdsp_fft_spec.h STFT section):
        //   S = Z[k] + conj(Z[M-k]),  D' = (Z[k].im + Z[M-k].im, -(Z[k].re - Z[M-k].re)),
        //   Y = S + rt[k] D' (FMA form),  |X[k]| = 2^-33 sqrt(fma(Y.re, Y.re, Y.im Y.im)) (the window carries
        //   2^32, so Y = 2^33 X);  bin M-k from the
        //   same S, D' conjugated with rt[M-k] = (-rt[k].re, rt[k].im).
        float* out = mags + (mag_row0[trk] + f) * (uint64_t)stride;
        float mx = 0.0f;
        uint32_t lo = 0xFFFFFFFFu, hi = 0u;
        auto sq = [&](float yx, float yy) { return 0x1p-33f * sqrt_fast(__builtin_fmaf(yx, yx, yy * yy), lo, hi); };
        // frame maximum: magnitudes are +0 or positive, so v_max_f32 (IEEE maxNum: a NaN operand
        // yields the other) is sd_maxf here except for the payload of an all-NaN row
        auto put = [&](int k, float mag) {
            out[k] = mag;
            if (FRAME_MAX) mx = __builtin_fmaxf(mx, mag);
        };
        // one pair: own bin k from Zk, partner bin M-k from Zr, post twiddle w = rt[k]
        auto pair = [&](c2 Zk, c2 Zr, c2 w, int k) {
            const float sx = Zk.x + Zr.x, sy = Zk.y - Zr.y, dx = Zk.y + Zr.y, dy = -(Zk.x - Zr.x);
            put(k, sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))));
            put(M - k, sq(__builtin_fmaf(-w.x, dx, __builtin_fmaf(w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, -sy))));
        };
        auto single = [&](c2 Z, c2 w, int k) {  // a self-paired bin (k = M/2)
            const float sx = Z.x + Z.x, sy = Z.y - Z.y, dx = Z.y + Z.y, dy = -(Z.x - Z.x);
            put(k, sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))));
        };
        if constexpr (M == 4096) {
            // pass 3 (n = 16, s = 256, p' = 0) on column colA: v[m] = Z[colA + 256 m]
            const int rb = lpad(colA);
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = bufB[rb + P272 * k];
            radix16<true>(v, tw3);
            // exchange: every lane sends its elements 8..15 to the partner lane (ds_bpermute);
            // the column-0 lane sends itself elements 9..15, 0 (its pairs are (m, 16 - m))
            c2 rv[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const c2 snd = self0 ? v[(9 + i) & 15] : v[8 + i];
                rv[i] = {__shfl(snd.x, src_lane, 64), __shfl(snd.y, src_lane, 64)};
            }
            // pair j: Z[colA + 256 j] with the partner column's element 15 - j (= rv[7 - j])
#pragma unroll
            for (int j = 0; j < 8; j++) pair(v[j], rv[7 - j], wk[j], colA + 256 * j);
            if (self0) single(v[8], rtH, M / 2);
        } else {
            // trailing radix-4 (n = 4, s = M/4, p = 0) on the thread's four columns
            c2 A[4], A2[4], Bv[4], B2[4];
            auto col4 = [&](int c, c2 (&z)[4]) {
                const int b = lpad(c);
                bfly4<false>(bufB[b], bufB[b + P272], bufB[b + 2 * P272], bufB[b + 3 * P272], c2{}, c2{}, c2{}, z[0],
                             z[1], z[2], z[3]);
            };
            col4(colA, A);
            col4(colA2, A2);
            col4(colB, Bv);
            col4(colB2, B2);
            // pairs of (colA, colA2): (A[j], A2[3 - j]); thread 0 (columns 0 and 128, each self-paired):
            // (A0, A0) -> bins 0 / M, (A1, A3) -> 256 / 768, (A2'0, A2'3) -> 128 / 896, (A2'1, A2'2) -> 384 / 640
            const c2 zk0 = A[0], zr0 = self0 ? A[0] : A2[3];
            const c2 zk1 = A[1], zr1 = self0 ? A[3] : A2[2];
            const c2 zk2 = self0 ? A2[0] : A[2], zr2 = self0 ? A2[3] : A2[1];
            const c2 zk3 = self0 ? A2[1] : A[3], zr3 = self0 ? A2[2] : A2[0];
            pair(zk0, zr0, wk[0], self0 ? 0 : colA);
            pair(zk1, zr1, wk[1], self0 ? 256 : colA + 256);
            pair(zk2, zr2, wk[2], self0 ? 128 : colA + 512);
            pair(zk3, zr3, wk[3], self0 ? 384 : colA + 768);
#pragma unroll
            for (int j = 0; j < 4; j++) pair(Bv[j], B2[3 - j], wk[4 + j], colB + 256 * j);
            if (self0) single(A[2], rtH, M / 2);
        }
        // a magnitude^2 of subnormal scale (or inf / NaN) somewhere in the frame: the frame goes on
        // the redo list, which k_stft_mag recomputes with the general sqrt right after this kernel
        // (stream order), overwriting the whole row.  Each frame is listed at most once, so the
        // list never holds more entries than the launch has frames: one wave per frame (N = 2048)
        // appends directly; the 4 waves of an 8192-point frame OR a flag in LDS, which thread 0
        // reads after the next frame's first barrier (or after the strip) and appends.
        const bool missed = __builtin_amdgcn_ballot_w64(sqrt_fast_missed(lo, hi)) != 0;
        if constexpr (TPF == 64) {
            if (__builtin_expect(missed, 0) && lt == 0) redo[1 + atomicAdd(redo, 1u)] = (uint32_t)(frame_pfx[trk] + f);
        } else {
            if (__builtin_expect(missed, 0) && (threadIdx.x & 63) == 0) atomicOr(&miss_flag[i & 1], 1u);
        }
        if constexpr (FRAME_MAX) {
            static_assert(!FRAME_MAX || TPF == 64, "frame maxima: one wave per frame");
            mx = wave_max(mx);
            if (lt == 0) frame_max[mag_row0[trk] + f] = mx;
        }
        // slide the ring
#pragma unroll
        for (int k = 0; k < 16 - S; k++) ring[k] = ring[k + S];
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) ring[16 - S + s2] = {nxt[s2].x * gn, nxt[s2].y * gn};
    }
    if constexpr (TPF == 256) {  // the strip's last frame
        __syncthreads();
        if (threadIdx.x == 0 && miss_flag[(nf - 1) & 1]) redo[1 + atomicAdd(redo, 1u)] = (uint32_t)(frame_pfx[trk] + f0 + nf - 1);
    }
}

// ---------------------------------------------------------------------------------------------
// k_stft_slide2s: the sliding strip for N = 2048 (M = 1024, one wave per strip, 4 strips per
// workgroup) with ONE frame buffer per strip and the pass-2 / post twiddles in LDS, for 3 waves
// per SIMD (k_stft_slide<2048>: two buffers per strip, 227 VGPRs, 2 waves).  Pass 2 runs in place:
// a thread reads its 16 slots and writes its 16 results back into them (a wave's LDS operations
// run in issue order, so no barrier), so z[q + 256 pp + 16 k] lives where x[q + 16 pp + 64 k] was
// read, and the trailing radix-4 reads column c, Z[c + 256 j], from (c % 16) + 68 (c / 16) + 17 j.
// Same arithmetic as k_stft_slide (bit-identical magnitudes and frame maxima).
template <int S, bool FRAME_MAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_stft_slide2s(
    const float* __restrict__ samples, const uint64_t* __restrict__ frame_pfx, const uint64_t* __restrict__ strip_pfx,
    int n_tracks, uint64_t n_strips, const uint64_t* __restrict__ src_off, const float* __restrict__ gain, int hop,
    const float* __restrict__ window, const cx* __restrict__ twp, const cx* __restrict__ rtp, float* __restrict__ mags,
    const uint64_t* __restrict__ mag_row0, int stride, float* __restrict__ frame_max, uint32_t* __restrict__ redo) {
    constexpr int M = 1024, TPF = 64, FPB = 4;
    constexpr int PADM = M + PADSHIFT * M / 16;  // 1088 slots
    static_assert(S >= 1 && S <= 16, "hop = S * 128");
    __shared__ c2 lds[FPB * PADM];
    __shared__ __attribute__((aligned(16))) c2 tw2s[4 * 16];  // [p'][j], j < 15
    __shared__ c2 wks[8 * TPF];                                // [slot j][lane]

    const int lt = threadIdx.x % TPF;
    const int fl = threadIdx.x / TPF;
    const __amdgpu_buffer_rsrc_t rtw = rsrc_of(twp, 8u * 15u * (TPF + TPF / 16 + 1));
    const __amdgpu_buffer_rsrc_t rrt = rsrc_of(rtp, 8u * (slide_rt_base<M>() + 8 * TPF + 1));
    // the workgroup's tables (every wave of the workgroup reaches this barrier)
    {
        const int j = threadIdx.x / TPF * 2, l = threadIdx.x % TPF;  // 256 threads: 2 of the 8 slots each
        wks[j * TPF + l] = ld_c2(rrt, 8 * l, 8 * (slide_rt_base<M>() + TPF * j));
        wks[(j + 1) * TPF + l] = ld_c2(rrt, 8 * l, 8 * (slide_rt_base<M>() + TPF * (j + 1)));
    }
    if (threadIdx.x < 4 * 15) {
        const int pp = threadIdx.x / 15, j = threadIdx.x % 15;
        tw2s[pp * 16 + j] = ld_c2(rtw, 8 * (15 * TPF + j * (TPF / 16) + pp), 0);
    }
    __syncthreads();
    const uint64_t strip =
        (uint64_t)__builtin_amdgcn_readfirstlane((int)((uint64_t)xcd_block(blockIdx.x, gridDim.x) * FPB + fl));
    if (strip >= n_strips) return;  // a whole wave
    const int trk = find_track(strip_pfx, n_tracks, strip);
    const uint64_t F = frame_pfx[trk + 1] - frame_pfx[trk];
    const uint64_t f0 = (strip - strip_pfx[trk]) * (uint64_t)STRIP_T;
    const int nf = (int)(F - f0 < (uint64_t)STRIP_T ? F - f0 : (uint64_t)STRIP_T);
    const float gn = gain[trk];
    c2* buf = lds + fl * PADM;
    const int vo = 8 * lt;
    const uint64_t cstart = f0 * (uint64_t)(hop / 2);
    const uint64_t clen = (uint64_t)(nf - 1) * (uint64_t)(hop / 2) + (uint64_t)M;
    const __amdgpu_buffer_rsrc_t rx = rsrc_of(samples + src_off[trk] + 2 * cstart, (uint32_t)(8u * clen));
    const __amdgpu_buffer_rsrc_t rw = rsrc_of(window, 4u * 2048u);

    c2 win[16], tw1[15], ring[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const c2 x = ld_c2(rx, vo, 8 * TPF * k);
        ring[k] = {x.x * gn, x.y * gn};
    }
#pragma unroll
    for (int k = 0; k < 16; k++) win[k] = ld_c2(rw, vo, 8 * TPF * k);
#pragma unroll
    for (int j = 0; j < 15; j++) tw1[j] = ld_c2(rtw, vo, 8 * TPF * j);
    const cx rth = rtp[slide_rt_base<M>() + 8 * TPF];  // bin M/2 (wave-uniform)
    const c2 rtH = {rth.re, rth.im};
    const int pp2 = lt / 16, q2 = lt % 16;
    int colA, colA2, colB, colB2;
    slide_cols2(lt, &colA, &colA2, &colB, &colB2);
    const bool self0 = lt == 0;
    // pass-1 stores at 17 lt + k; pass 2 in place at q + 17 pp + 68 k; column c at (c % 16) + 68 (c / 16) + 17 j
    const int rb2 = q2 + 17 * pp2;
    auto colbase = [](int c) { return (c & 15) + 68 * (c >> 4); };
    // store byte offsets in a row (bins above, M = 1024): partner offsets are based at the slot
    // with the largest scalar offset so every scalar part is >= 0
    const int vA = 4 * colA, vAr = 4 * (M - colA - 768);
    const int vA2 = 4 * (self0 ? 128 : colA + 512), vA2r = 4 * (M - (self0 ? 128 : colA + 512));
    const int vA3 = 4 * (self0 ? 384 : colA + 768), vA3r = 4 * (M - (self0 ? 384 : colA + 768));
    const int vB = 4 * colB, vBr = 4 * (M - colB - 768);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the per-strip loads have landed

    for (int i = 0; i < nf; i++) {
        const uint64_t f = f0 + (uint64_t)i;
        c2 nxt[S];
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) nxt[s2] = ld_c2(rx, vo, 8 * ((i + 1) * (hop / 2) + TPF * (16 - S + s2)));
        c2 v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = {ring[k].x * win[k].x, ring[k].y * win[k].y};
        radix16<false>(v, tw1);
        frame_sync<TPF>();  // the previous frame's column reads are done (in-order LDS)
#pragma unroll
        for (int k = 0; k < 16; k++) buf[P17 * lt + k] = v[k];
        frame_sync<TPF>();
        // pass 2 (n = M/16 = 64, s = 16), in place
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = buf[rb2 + 68 * k];
        radix16_tw(v, [&](int j) { return tw2s[pp2 * 16 + j]; });
#pragma unroll
        for (int k = 0; k < 16; k++) buf[rb2 + 68 * k] = v[k];
        frame_sync<TPF>();
        // the frame's row as a buffer resource: per-lane byte offsets fixed for the strip, the
        // slot's bin offset a scalar constant (no 64-bit address arithmetic per store)
        const __amdgpu_buffer_rsrc_t ro = rsrc_of(mags + (mag_row0[trk] + f) * (uint64_t)stride, 4u * (M + 1));
        float mx = 0.0f;
        uint32_t lo = 0xFFFFFFFFu, hi = 0u;
        auto sq = [&](float yx, float yy) { return 0x1p-33f * sqrt_fast(__builtin_fmaf(yx, yx, yy * yy), lo, hi); };
        auto put = [&](int voff, int soff, float mag) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mag), ro, voff, soff, 0);
            if (FRAME_MAX) mx = __builtin_fmaxf(mx, mag);
        };
        // own bin at (vk, sk), partner bin M - k at (vr, sr)
        auto pair = [&](c2 Zk, c2 Zr, c2 w, int vk, int sk, int vr, int sr) {
            const float sx = Zk.x + Zr.x, sy = Zk.y - Zr.y, dx = Zk.y + Zr.y, dy = -(Zk.x - Zr.x);
            put(vk, sk, sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))));
            put(vr, sr, sq(__builtin_fmaf(-w.x, dx, __builtin_fmaf(w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, -sy))));
        };
        auto single = [&](c2 Z, c2 w, int k) {
            const float sx = Z.x + Z.x, sy = Z.y - Z.y, dx = Z.y + Z.y, dy = -(Z.x - Z.x);
            put(0, 4 * k, sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))));
        };
        // trailing radix-4 (n = 4, s = M/4, p = 0) on the thread's four columns
        c2 A[4], A2[4], Bv[4], B2[4];
        auto col4 = [&](int c, c2 (&z)[4]) {
            const int b = colbase(c);
            bfly4<false>(buf[b], buf[b + 17], buf[b + 34], buf[b + 51], c2{}, c2{}, c2{}, z[0], z[1], z[2], z[3]);
        };
        col4(colA, A);
        col4(colA2, A2);
        col4(colB, Bv);
        col4(colB2, B2);
        const c2 zk0 = A[0], zr0 = self0 ? A[0] : A2[3];
        const c2 zk1 = A[1], zr1 = self0 ? A[3] : A2[2];
        const c2 zk2 = self0 ? A2[0] : A[2], zr2 = self0 ? A2[3] : A2[1];
        const c2 zk3 = self0 ? A2[1] : A[3], zr3 = self0 ? A2[2] : A2[0];
        // bins (k, M - k): colA + 256 j for j < 2 (thread 0: 0 / 1024, 256 / 768 as well), then
        // colA + 512, colA + 768 (thread 0: 128 / 896, 384 / 640); colB + 256 j for the B pairs
        pair(zk0, zr0, wks[0 * TPF + lt], vA, 0, vAr, 3 * 1024);
        pair(zk1, zr1, wks[1 * TPF + lt], vA, 1024, vAr, 2 * 1024);
        pair(zk2, zr2, wks[2 * TPF + lt], vA2, 0, vA2r, 0);
        pair(zk3, zr3, wks[3 * TPF + lt], vA3, 0, vA3r, 0);
#pragma unroll
        for (int j = 0; j < 4; j++) pair(Bv[j], B2[3 - j], wks[(4 + j) * TPF + lt], vB, 1024 * j, vBr, 1024 * (3 - j));
        if (self0) single(A[2], rtH, M / 2);
        const bool missed = __builtin_amdgcn_ballot_w64(sqrt_fast_missed(lo, hi)) != 0;
        if (__builtin_expect(missed, 0) && lt == 0) redo[1 + atomicAdd(redo, 1u)] = (uint32_t)(frame_pfx[trk] + f);
        if constexpr (FRAME_MAX) {
            mx = wave_max(mx);
            if (lt == 0) frame_max[mag_row0[trk] + f] = mx;
        }
#pragma unroll
        for (int k = 0; k < 16 - S; k++) ring[k] = ring[k + S];
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) ring[16 - S + s2] = {nxt[s2].x * gn, nxt[s2].y * gn};
    }
}

// ---------------------------------------------------------------------------------------------
// k_stft_slide8: the sliding strip for N = 8192 (M = 4096 = 16^3, one 256-thread workgroup per
// strip), software-pipelined across frames.  The kernel holds its per-strip constants in ~110
// VGPRs, so it runs 2 waves per SIMD, and one wave alone issues a VALU instruction at most every
// 4 cycles (MI355X_MICROARCH.md, issue costs): the SIMD reaches its 2-cycle rate only while both
// of its waves issue VALU.  Every LDS round trip is therefore given independent VALU work of
// another frame to cover its latency:
//   region 1 (after the barrier that publishes frame i's pass-1 output in A):
//       issue frame i's pass-2 reads from A; post-process frame i-1 (held in registers: S, D',
//       the FMA form, the exact sqrt, 16 buffer stores); pass 2 of frame i; write B;
//   barrier;
//   region 2: issue frame i's pass-3 reads from B; window + pass 1 of frame i+1 from the sample
//       ring, write A (every pass-2 read of A finished before the barrier); pass 3 of frame i; the
//       (k, M-k) exchange between lanes l and l^32 (ds_bpermute) into the held registers;
//   barrier (A complete for frame i+1; every pass-3 read of B done before the next B write).
// Two barriers per frame, as before, and the same arithmetic (bit-identical magnitudes).  Rows
// are written by buffer stores whose per-lane offsets are fixed for the strip and whose row is a
// scalar descriptor (no 64-bit address arithmetic per store); the descriptor of the row "before
// frame 0" has no records, so its stores are dropped by the hardware without a branch.  Frames
// whose sqrt met an input outside its exact range are collected in a wave-uniform 64-bit mask and
// listed once per strip after the loop (no per-frame LDS flag).
template <int S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_stft_slide8(
    const float* __restrict__ samples, const uint64_t* __restrict__ frame_pfx, const uint64_t* __restrict__ strip_pfx,
    int n_tracks, uint64_t n_strips, const uint64_t* __restrict__ src_off, const float* __restrict__ gain, int hop,
    const float* __restrict__ window, const cx* __restrict__ twp, const cx* __restrict__ rtp, float* __restrict__ mags,
    const uint64_t* __restrict__ mag_row0, int stride, uint32_t* __restrict__ redo) {
    constexpr int M = 4096, TPF = 256;
    constexpr int PADM = M + PADSHIFT * M / 16;
    static_assert(S >= 1 && S <= 16 && STRIP_T == 64, "hop = S * 512; the miss mask holds 64 frames");
    __shared__ c2 lds[2 * PADM];
    __shared__ uint64_t miss_mask[4];

    const int lt = threadIdx.x;
    const uint64_t strip = (uint64_t)__builtin_amdgcn_readfirstlane((int)xcd_block(blockIdx.x, gridDim.x));
    if (strip >= n_strips) return;  // the whole workgroup
    const int trk = find_track(strip_pfx, n_tracks, strip);
    const uint64_t F = frame_pfx[trk + 1] - frame_pfx[trk];
    const uint64_t f0 = (strip - strip_pfx[trk]) * (uint64_t)STRIP_T;
    const int nf = (int)(F - f0 < (uint64_t)STRIP_T ? F - f0 : (uint64_t)STRIP_T);
    const float gn = gain[trk];
    c2* const bufA = lds;
    c2* const bufB = lds + PADM;
    const int vo = 8 * lt;
    const uint64_t cstart = f0 * (uint64_t)(hop / 2);
    const uint64_t clen = (uint64_t)(nf - 1) * (uint64_t)(hop / 2) + (uint64_t)M;
    const __amdgpu_buffer_rsrc_t rx = rsrc_of(samples + src_off[trk] + 2 * cstart, (uint32_t)(8u * clen));
    const __amdgpu_buffer_rsrc_t rw = rsrc_of(window, 4u * 8192u);
    const __amdgpu_buffer_rsrc_t rtw = rsrc_of(twp, 8u * 15u * (TPF + TPF / 16 + 1));
    const __amdgpu_buffer_rsrc_t rrt = rsrc_of(rtp, 8u * (slide_rt_base<M>() + 8 * TPF + 1));
    float* const row0 = mags + (mag_row0[trk] + f0) * (uint64_t)stride;

    // per-strip constants (as k_stft_slide)
    c2 win[16], tw1[15], tw2[15], tw3[15], wk[8], ring[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const c2 x = ld_c2(rx, vo, 8 * TPF * k);
        ring[k] = {x.x * gn, x.y * gn};
    }
#pragma unroll
    for (int k = 0; k < 16; k++) win[k] = ld_c2(rw, vo, 8 * TPF * k);
#pragma unroll
    for (int j = 0; j < 15; j++) tw1[j] = ld_c2(rtw, vo, 8 * TPF * j);
    const int pp2 = lt / 16, q2 = lt % 16;
#pragma unroll
    for (int j = 0; j < 15; j++) tw2[j] = ld_c2(rtw, 8 * pp2, 8 * (15 * TPF + j * (TPF / 16)));
#pragma unroll
    for (int j = 0; j < 8; j++) wk[j] = ld_c2(rrt, vo, 8 * (slide_rt_base<M>() + TPF * j));
#pragma unroll
    for (int j = 0; j < 15; j++) {
        const cx t = twp[15 * TPF + 15 * (TPF / 16) + j];
        tw3[j] = c2{t.re, t.im};
    }
    const c2 rtH = ld_c2(rrt, 0, 8 * (slide_rt_base<M>() + 8 * TPF));  // bin M/2
    const int colA = slide_col8(lt);
    const bool self0 = lt == 0, self128 = lt == 32;
    const int src_lane = (self0 || self128) ? (lt & 63) : ((lt & 63) ^ 32);
    // LDS bases: pass-2 reads x[q + 16 pp + 256 k] (lpad: + 272 k), writes z[q + 256 pp + 16 k] (+ 17 k);
    // pass-3 reads column colA, Z[colA + 256 m] (+ 272 m)
    const int rb2 = lpad(q2 + 16 * pp2), wb2 = q2 + P272 * pp2, rb3 = lpad(colA);
    // byte offsets in a row: own bins colA + 256 j, partner bins M - colA - 256 j
    const int vown = 4 * colA, vpart = 4 * (M - colA - 256 * 7), vmid = 4 * (M / 2);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the per-strip loads have landed

    // prologue: pass 1 of frame 0 into A, the ring advanced to frame 1
    c2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = {ring[k].x * win[k].x, ring[k].y * win[k].y};
    radix16<false>(v, tw1);
#pragma unroll
    for (int k = 0; k < 16; k++) bufA[P17 * lt + k] = v[k];
    {
        c2 nx[S];
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) nx[s2] = ld_c2(rx, vo, 8 * ((hop / 2) + TPF * (16 - S + s2)));
#pragma unroll
        for (int k = 0; k < 16 - S; k++) ring[k] = ring[k + S];
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) ring[16 - S + s2] = {nx[s2].x * gn, nx[s2].y * gn};
    }
    __syncthreads();

    // the held frame (i - 1): P[0..7] own Z[colA + 256 j], P[8..15] the partner column's elements
    // 8..15 (received), Pm = own element 8 (bin M/2 on the column-0 lane)
    c2 P[16], Pm = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 16; k++) P[k] = {0.0f, 0.0f};
    uint64_t miss = 0;  // wave-uniform: bit i = frame f0 + i met the sqrt's inexact range
    for (int i = 0;; i++) {
        // ---- region 1 ----
        c2 nx[S];  // the ring's new values for frame i + 2 (zeros past the strip: outside rx)
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) nx[s2] = ld_c2(rx, vo, 8 * ((i + 2) * (hop / 2) + TPF * (16 - S + s2)));
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = bufA[rb2 + P272 * k];
        __builtin_amdgcn_sched_barrier(0);  // the reads first: the post-processing below covers their latency
        {
            // post-processing of frame i - 1 (sdsp_fft_spec.h STFT section; see k_stft_slide)
            const bool live = i > 0;
            const __amdgpu_buffer_rsrc_t ro = rsrc_of(row0 + (int64_t)(i - 1) * stride, live ? 4u * (M + 1) : 0u);
            uint32_t lo = 0xFFFFFFFFu, hi = 0u;
            // |X| = 2^-33 sqrt(e) with the exact fast sqrt
            auto sq = [&](float yx, float yy) { return 0x1p-33f * sqrt_fast(__builtin_fmaf(yx, yx, yy * yy), lo, hi); };
            auto st = [&](float mag, int voff, int soff) {
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mag), ro, voff, soff, 0);
            };
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const c2 Zk = P[j], Zr = P[15 - j], w = wk[j];
                const float sx = Zk.x + Zr.x, sy = Zk.y - Zr.y, dx = Zk.y + Zr.y, dy = -(Zk.x - Zr.x);
                st(sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))),
                   vown, 1024 * j);
                st(sq(__builtin_fmaf(-w.x, dx, __builtin_fmaf(w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, -sy))),
                   vpart, 1024 * (7 - j));
            }
            if (self0) {  // bin M/2, self-paired
                const c2 Z = Pm, w = rtH;
                const float sx = Z.x + Z.x, sy = Z.y - Z.y, dx = Z.y + Z.y, dy = -(Z.x - Z.x);
                st(sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))),
                   vmid, 0);
            }
            const bool missed = __builtin_amdgcn_ballot_w64(sqrt_fast_missed(lo, hi)) != 0;
            miss |= (uint64_t)(missed && live) << ((i - 1) & 63);
        }
        if (i == nf) break;
        radix16<false>(v, tw2);
#pragma unroll
        for (int k = 0; k < 16; k++) bufB[wb2 + P17 * k] = v[k];
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);  // keep region 2's VALU below the barrier (it covers the pass-3 reads)
        // ---- region 2 ----
        c2 u[16];
#pragma unroll
        for (int k = 0; k < 16; k++) u[k] = bufB[rb3 + P272 * k];
        __builtin_amdgcn_sched_barrier(0);  // the reads first: pass 1 below covers their latency
        // pass 1 of frame i + 1 (past the strip's end: unused values into A, nothing reads them)
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = {ring[k].x * win[k].x, ring[k].y * win[k].y};
        radix16<false>(v, tw1);
#pragma unroll
        for (int k = 0; k < 16; k++) bufA[P17 * lt + k] = v[k];
#pragma unroll
        for (int k = 0; k < 16 - S; k++) ring[k] = ring[k + S];
#pragma unroll
        for (int s2 = 0; s2 < S; s2++) ring[16 - S + s2] = {nx[s2].x * gn, nx[s2].y * gn};
        // pass 3 of frame i (n = 16, s = 256, p' = 0) on column colA, then the exchange: every lane
        // sends its elements 8..15 to the partner lane; the column-0 lane sends itself 9..15, 0
        radix16<true>(u, tw3);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const c2 snd = self0 ? u[(9 + k) & 15] : u[8 + k];
            P[8 + k] = {__shfl(snd.x, src_lane, 64), __shfl(snd.y, src_lane, 64)};
            P[k] = u[k];
        }
        Pm = u[8];
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);  // keep the post-processing below the barrier (it covers the pass-2 reads)
    }
    // list the strip's missed frames once (k_stft_mag recomputes them right after this kernel)
    if ((lt & 63) == 0) miss_mask[lt >> 6] = miss;
    __syncthreads();
    if (lt == 0) {
        uint64_t m = miss_mask[0] | miss_mask[1] | miss_mask[2] | miss_mask[3];
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            redo[1 + atomicAdd(redo, 1u)] = (uint32_t)(frame_pfx[trk] + f0 + (uint64_t)b);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// k_stft_slide8w3: the sliding strip for N = 8192 at 3 waves per SIMD (3 workgroups per CU; the
// budget is <= 168 VGPRs and <= 53 KB of LDS per 256-thread workgroup).  k_stft_slide8 runs 2
// waves per SIMD (229 VGPRs, two 34.8 KB frame buffers), and one wave issues a VALU instruction
// at most every 4 cycles, so the SIMD's VALU idles whenever either wave waits.
// What moves to fit the budget, the arithmetic unchanged (bit-identical magnitudes):
//  * ONE frame buffer, pass 2 in place: a pass-2 thread reads its 16 slots, runs the radix-16
//    pass and writes the 16 results back into the same slots (the threads' slot sets are
//    disjoint, so no barrier between its reads and its writes).  Element z[q + 256 pp + 16 k]
//    then lives where x[q + 16 pp + 256 k] was read, and the last pass reads column c, Z[c + 256 m],
//    from slots (c % 16) + 272 (c / 16) + 17 m: conflict-free for ds_read_b64 on every lane;
//  * a third barrier per frame, before the next frame's pass-1 stores (its pass-1 arithmetic runs
//    before that barrier, from the register ring, while other workgroups of the CU issue);
//  * the pass-2 twiddles (16 p' x 15, 1.9 KB, four distinct p' per wave: broadcast reads) and the
//    post twiddles (8 slots x 256 lanes, 16 KB) from LDS instead of 46 VGPRs; the pass-3
//    twiddles stay wave-uniform scalars; window, pass-1 twiddles and the sample ring stay in VGPRs.
template <int S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_stft_slide8w3(
    const float* __restrict__ samples, const uint64_t* __restrict__ frame_pfx, const uint64_t* __restrict__ strip_pfx,
    int n_tracks, uint64_t n_strips, const uint64_t* __restrict__ src_off, const float* __restrict__ gain, int hop,
    const float* __restrict__ window, const cx* __restrict__ twp, const cx* __restrict__ rtp, float* __restrict__ mags,
    const uint64_t* __restrict__ mag_row0, int stride, uint32_t* __restrict__ redo) {
    constexpr int M = 4096, TPF = 256;
    constexpr int PADM = M + PADSHIFT * M / 16;
    static_assert(S >= 1 && S <= 16 && STRIP_T == 64, "hop = S * 512; the miss mask holds 64 frames");
    __shared__ c2 buf[PADM];
    __shared__ __attribute__((aligned(16))) c2 tw2s[16 * 16];  // [p'][j], j < 15
    __shared__ c2 wks[8 * TPF];                                 // [slot j][lane]
    __shared__ uint64_t miss_mask[4];

    const int lt = threadIdx.x;
    const uint64_t strip = (uint64_t)__builtin_amdgcn_readfirstlane((int)xcd_block(blockIdx.x, gridDim.x));
    if (strip >= n_strips) return;  // the whole workgroup
    const int trk = find_track(strip_pfx, n_tracks, strip);
    const uint64_t F = frame_pfx[trk + 1] - frame_pfx[trk];
    const uint64_t f0 = (strip - strip_pfx[trk]) * (uint64_t)STRIP_T;
    const int nf = (int)(F - f0 < (uint64_t)STRIP_T ? F - f0 : (uint64_t)STRIP_T);
    const float gn = gain[trk];
    const int vo = 8 * lt;
    const uint64_t cstart = f0 * (uint64_t)(hop / 2);
    const uint64_t clen = (uint64_t)(nf - 1) * (uint64_t)(hop / 2) + (uint64_t)M;
    const __amdgpu_buffer_rsrc_t rx = rsrc_of(samples + src_off[trk] + 2 * cstart, (uint32_t)(8u * clen));
    const __amdgpu_buffer_rsrc_t rw = rsrc_of(window, 4u * 8192u);
    const __amdgpu_buffer_rsrc_t rtw = rsrc_of(twp, 8u * 15u * (TPF + TPF / 16 + 1));
    const __amdgpu_buffer_rsrc_t rrt = rsrc_of(rtp, 8u * (slide_rt_base<M>() + 8 * TPF + 1));
    float* const row0 = mags + (mag_row0[trk] + f0) * (uint64_t)stride;

    // LDS tables (published by the first frame's first barrier)
#pragma unroll
    for (int j = 0; j < 8; j++) wks[j * TPF + lt] = ld_c2(rrt, vo, 8 * (slide_rt_base<M>() + TPF * j));
    if (lt < 15 * 16) {
        const int pp = lt / 15, j = lt % 15;
        tw2s[pp * 16 + j] = ld_c2(rtw, 8 * (15 * TPF + j * (TPF / 16) + pp), 0);
    }
    // per-strip register constants: window, pass-1 twiddles, the sample ring; pass 3 wave-uniform.
    // At hop 512 (S = 1) the frame loop is unrolled by U = 2 frames, so the ring holds 16 + S
    // entries and shifts by 2 S once per two frames (16 - S moves of a complex value per two frames
    // instead of per frame); at S = 2 the two-frame ring would spill, so U = 1.
    // ring[k] = x[TPF ((f + 1) S + k) + lt] * gain at the top of an iteration starting at frame f.
    constexpr int U = S == 1 ? 2 : 1, RN = 16 + (U - 1) * S;
    c2 win[16], tw1[15], tw3[15], ring[RN];
#pragma unroll
    for (int k = 0; k < RN; k++) {
        const c2 x = ld_c2(rx, vo, 8 * TPF * (S + k));
        ring[k] = {x.x * gn, x.y * gn};
    }
#pragma unroll
    for (int k = 0; k < 16; k++) win[k] = ld_c2(rw, vo, 8 * TPF * k);
#pragma unroll
    for (int j = 0; j < 15; j++) tw1[j] = ld_c2(rtw, vo, 8 * TPF * j);
#pragma unroll
    for (int j = 0; j < 15; j++) {
        const cx t = twp[15 * TPF + 15 * (TPF / 16) + j];
        tw3[j] = c2{t.re, t.im};
    }
    const cx rth = rtp[slide_rt_base<M>() + 8 * TPF];  // bin M/2 (wave-uniform: scalar)
    const c2 rtH = {rth.re, rth.im};
    const int pp2 = lt / 16, q2 = lt % 16;
    const int colA = slide_col8(lt);
    const bool self0 = lt == 0, self128 = lt == 32;
    const int src_lane = (self0 || self128) ? (lt & 63) : ((lt & 63) ^ 32);
    // slots: pass-1 stores 17 lt + k; pass 2 reads and writes back q + 17 pp + 272 k; the last
    // pass reads (c % 16) + 272 (c / 16) + 17 m for its column c
    const int rb2 = q2 + 17 * pp2, rb3 = (colA & 15) + P272 * (colA >> 4);
    const int vown = 4 * colA, vpart = 4 * (M - colA - 256 * 7), vmid = 4 * (M / 2);

    // prologue: pass 1 of frame 0 in registers (its samples x[TPF k + lt], k < 16)
    c2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const c2 x = ld_c2(rx, vo, 8 * TPF * k);
        v[k] = {(x.x * gn) * win[k].x, (x.y * gn) * win[k].y};
    }
    radix16<false>(v, tw1);

    uint64_t miss = 0;  // wave-uniform: bit i = frame f0 + i met the sqrt's inexact range
    // frame i from v (its pass-1 output): LDS passes 2 and 3, the exchange, the post-processing
    auto frame = [&](int i) {
        if (i > 0) __syncthreads();  // every last-pass read of frame i - 1 is done
#pragma unroll
        for (int k = 0; k < 16; k++) {
            buf[P17 * lt + k] = v[k];
        }
        __syncthreads();
        // pass 2 (n = M/16, s = 16), in place
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = buf[rb2 + P272 * k];
        radix16_tw(v, [&](int j) { return tw2s[pp2 * 16 + j]; });
#pragma unroll
        for (int k = 0; k < 16; k++) buf[rb2 + P272 * k] = v[k];
        __syncthreads();
        // last pass (n = 16, s = 256, p' = 0) on column colA, then the (k, M-k) exchange between
        // lanes l and l^32: every lane sends its elements 8..15; the column-0 lane sends itself 9..15, 0
#ifndef SDSP_STFT8_PAIRED
        lds_ld16<P17>(&buf[rb3], v);
#else
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = buf[rb3 + P17 * k];
#endif
        radix16<true>(v, tw3);
        c2 P[16];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const c2 snd = self0 ? v[(9 + k) & 15] : v[8 + k];
            P[8 + k] = {__shfl(snd.x, src_lane, 64), __shfl(snd.y, src_lane, 64)};
            P[k] = v[k];
        }
        const c2 Pm = v[8];
        // post-processing of frame i (sdsp_fft_spec.h STFT section; see k_stft_slide)
        const __amdgpu_buffer_rsrc_t ro = rsrc_of(row0 + (int64_t)i * stride, 4u * (M + 1));
        uint32_t lo = 0xFFFFFFFFu, hi = 0u;
        auto sq = [&](float yx, float yy) { return 0x1p-33f * sqrt_fast(__builtin_fmaf(yx, yx, yy * yy), lo, hi); };
        auto st = [&](float mag, int voff, int soff) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mag), ro, voff, soff, 0);
        };
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const c2 Zk = P[j], Zr = P[15 - j], w = wks[j * TPF + lt];
            const float sx = Zk.x + Zr.x, sy = Zk.y - Zr.y, dx = Zk.y + Zr.y, dy = -(Zk.x - Zr.x);
            st(sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))),
               vown, 1024 * j);
            st(sq(__builtin_fmaf(-w.x, dx, __builtin_fmaf(w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, -sy))),
               vpart, 1024 * (7 - j));
        }
        if (self0) {  // bin M/2, self-paired
            const c2 Z = Pm, w = rtH;
            const float sx = Z.x + Z.x, sy = Z.y - Z.y, dx = Z.y + Z.y, dy = -(Z.x - Z.x);
            st(sq(__builtin_fmaf(w.x, dx, __builtin_fmaf(-w.y, dy, sx)), __builtin_fmaf(w.x, dy, __builtin_fmaf(w.y, dx, sy))),
               vmid, 0);
        }
        const bool missed = __builtin_amdgcn_ballot_w64(sqrt_fast_missed(lo, hi)) != 0;
        miss |= (uint64_t)missed << (i & 63);
    };
    // pass 1 of the next frame from ring[o .. o + 15] (stored after the next barrier)
    auto pass1 = [&](int o) {
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = {ring[o + k].x * win[k].x, ring[o + k].y * win[k].y};
        radix16<false>(v, tw1);
    };
    for (int i = 0;; i += U) {
        // the ring's U S new values for the next iteration (zeros past the strip: outside rx)
        c2 nx[U * S];
#pragma unroll
        for (int s2 = 0; s2 < U * S; s2++) nx[s2] = ld_c2(rx, vo, 8 * TPF * ((i + U + 1) * S + 16 - S + s2));
        frame(i);
        if (i + 1 == nf) break;
        pass1(0);
        if constexpr (U == 2) {
            frame(i + 1);
            if (i + 2 == nf) break;
            pass1(S);
        }
#pragma unroll
        for (int k = 0; k < 16 - S; k++) ring[k] = ring[k + U * S];
#pragma unroll
        for (int s2 = 0; s2 < U * S; s2++) ring[16 - S + s2] = {nx[s2].x * gn, nx[s2].y * gn};
    }
    // list the strip's missed frames once (k_stft_mag recomputes them right after this kernel)
    if ((lt & 63) == 0) miss_mask[lt >> 6] = miss;
    __syncthreads();
    if (lt == 0) {
        uint64_t m = miss_mask[0] | miss_mask[1] | miss_mask[2] | miss_mask[3];
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            redo[1 + atomicAdd(redo, 1u)] = (uint32_t)(frame_pfx[trk] + f0 + (uint64_t)b);
        }
    }
}

// strips of STRIP_T frames per track: strip_pfx[t] = sum over tracks < t of ceil(F / STRIP_T)
std::vector<uint64_t> stft_strips(const std::vector<uint64_t>& frame_pfx) {
    std::vector<uint64_t> sp(frame_pfx.size(), 0);
    for (size_t t = 0; t + 1 < frame_pfx.size(); t++)
        sp[t + 1] = sp[t] + (frame_pfx[t + 1] - frame_pfx[t] + STRIP_T - 1) / STRIP_T;
    return sp;
}

// Host: per-thread twiddle layouts for k_stft_mag, from the spec's tables (values unchanged).
//   twp[base(pass) + j (TPF/s) + p']: pass (n, s) = (M / 16^pass, 16^pass), p' = lt / s,
//       base(pass) = 15 sum_{q < pass} TPF / 16^q,
//       j = 3 j' + jA - 1 (< 12): tw[jA (p' + j' n/16) M/n];  j = 12 + jB - 1: tw[jB p' 4M/n]
//   rtp[(2 j + side) TPF + lt]: k = 1 + lt + TPF j (< M/2): side 0 rt[k], side 1 rt[M-k];
//   rtp[2 NPAIR TPF + {0,1,2,3}] = rt[0], rt[M], rt[M/2], tw[0]
void stft_tables(int N, const std::vector<float>& tw, const std::vector<float>& rt, std::vector<float>* twp,
                 std::vector<float>* rtp) {
    const int M = N / 2, TPF = M / 16;
    const int npass = M == 4096 ? 3 : M == 1024 ? 2 : 0;
    if (!npass) throw HipError("stft_tables: unsupported size");
    auto put = [](std::vector<float>* v, size_t i, const float* src) {
        (*v)[2 * i] = src[0];
        (*v)[2 * i + 1] = src[1];
    };
    static const float one[2] = {1.0f, 0.0f};  // a p = 0 twiddle: the FMA product is the operand
    size_t len = 0;
    for (int pass = 0, s = 1; pass < npass; pass++, s *= 16) len += (size_t)15 * (TPF / s);
    twp->assign(2 * len, 0.0f);
    size_t base = 0;
    for (int pass = 0, n = M, s = 1; pass < npass; pass++, n /= 16, s *= 16) {
        const int m1 = n / 16, tA = M / n, tB = 4 * (M / n), npp = TPF / s;
        for (int pp = 0; pp < npp; pp++) {
            for (int jp = 0; jp < 4; jp++)
                for (int ja = 1; ja <= 3; ja++)
                    put(twp, base + (size_t)(3 * jp + ja - 1) * npp + pp,
                        pp + jp * m1 == 0 ? one : &tw[2 * (size_t)(ja * (pp + jp * m1) * tA)]);
            for (int jb = 1; jb <= 3; jb++)
                put(twp, base + (size_t)(12 + jb - 1) * npp + pp, pp == 0 ? one : &tw[2 * (size_t)(jb * pp * tB)]);
        }
        base += (size_t)15 * npp;
    }
    const int npair = (M / 2 + TPF - 1) / TPF, sp = npair * 2 * TPF;
    rtp->assign((size_t)2 * (sp + 4), 0.0f);
    for (int j = 0; j < npair; j++)
        for (int lt = 0; lt < TPF; lt++) {
            const int k = 1 + lt + TPF * j;
            if (k >= M / 2) continue;
            put(rtp, (size_t)(2 * j) * TPF + lt, &rt[2 * (size_t)k]);
            // the STFT section's symmetric post twiddles: rt[M-k] = (-rt[k].re, rt[k].im)
            const float sym[2] = {-rt[2 * (size_t)k], rt[2 * (size_t)k + 1]};
            put(rtp, (size_t)(2 * j + 1) * TPF + lt, sym);
        }
    put(rtp, (size_t)sp + 0, &rt[0]);
    const float rtm[2] = {-rt[0], rt[1]};  // rt[M] := (-rt[0].re, rt[0].im), the symmetric rule at k = 0
    put(rtp, (size_t)sp + 1, rtm);
    put(rtp, (size_t)sp + 2, &rt[2 * (size_t)(M / 2)]);
    put(rtp, (size_t)sp + 3, &tw[0]);
    // k_stft_slide's post table: [slot j < 8][lane] = rt of the slot's own bin (slide_bin), then
    // rt[M/2]; bins above M/2 take the symmetric value (-rt[M-k].re, rt[M-k].im)
    const size_t sbase = (size_t)sp + 4;
    rtp->resize(2 * (sbase + 8 * (size_t)TPF + 1), 0.0f);
    for (int j = 0; j < 8; j++)
        for (int lt = 0; lt < TPF; lt++) {
            const int k = slide_bin(M, lt, j);
            const float v[2] = {k <= M / 2 ? rt[2 * (size_t)k] : -rt[2 * (size_t)(M - k)],
                                k <= M / 2 ? rt[2 * (size_t)k + 1] : rt[2 * (size_t)(M - k) + 1]};
            put(rtp, sbase + (size_t)j * TPF + lt, v);
        }
    put(rtp, sbase + 8 * (size_t)TPF, &rt[2 * (size_t)(M / 2)]);
}

bool stft_tuned(int N) { return N == 2048 || N == 8192; }
bool stft_size_ok(int N) { return N >= STFT_GEN_MIN && N <= STFT_GEN_MAX && (N & (N - 1)) == 0; }

// hop = S * 2 * TPF complex values with a k_stft_slide instance
bool stft_slide_ok(int nfft, int hop) {
    if (nfft == 8192) return hop == 512 || hop == 1024;
    if (nfft == 2048) return hop == 256 || hop == 512 || hop == 1024;
    return false;
}

// host launcher (the runtime owns all buffers; see runtime.hip).  With strip_pfx (stft_strips of
// the frame prefix, on the device) and a hop stft_slide_ok accepts, the sliding-strip kernel runs;
// otherwise the frame-parallel one.
void launch_stft(int nfft, bool frame_max, const float* samples, const uint64_t* frame_pfx, int n_tracks,
                 uint64_t total_frames, const uint64_t* src_off, const float* gain, int hop, const float* window,
                 const cx* twp, const cx* rtp, float* mags, const uint64_t* mag_row0, int stride, float* fmax,
                 hipStream_t st, const uint64_t* strip_pfx, uint64_t n_strips, uint32_t* redo) {
    if (total_frames == 0) return;
    const dim3 block(256);
    // the general kernel: other sizes, and N = 8192 with frame maxima (a tempo-path frame_size of
    // 8192; the tuned 8192 kernels serve the key path, which needs none)
    if (stft_general(nfft, frame_max)) {
        if (!stft_size_ok(nfft)) throw HipError("launch_stft: frame size not a power of two in [64, 16384]");
        if (total_frames > 0xffffffffull) throw HipError("launch_stft: too many frames for one launch");
        const size_t lds = (size_t)8 * (size_t)nfft;  // two buffers of N/2 complex values
        // set on every large launch: the attribute is per device, and several device workers may
        // launch at once (a process-wide "done" flag would race and skip the other devices)
        if (lds > 65536)
            SDSP_HIP_CHECK(hipFuncSetAttribute(frame_max ? (const void*)k_stft_gen<true> : (const void*)k_stft_gen<false>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(8 * STFT_GEN_MAX)));
        if (frame_max)
            hipLaunchKernelGGL(k_stft_gen<true>, dim3((unsigned)total_frames), block, lds, st, nfft, samples, frame_pfx,
                               n_tracks, total_frames, src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax);
        else
            hipLaunchKernelGGL(k_stft_gen<false>, dim3((unsigned)total_frames), block, lds, st, nfft, samples, frame_pfx,
                               n_tracks, total_frames, src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax);
        return;
    }
    if (strip_pfx && n_strips && redo && stft_slide_ok(nfft, hop)) {
        // redo[0] = 0; redo[1..] receives the frames the sliding kernel could not finish exactly
        SDSP_HIP_CHECK(hipMemsetAsync(redo, 0, sizeof(uint32_t), st));
#ifdef SDSP_STFT2_W2
#define SDSP_SLIDE(N, S, FM)                                                                                      \
    hipLaunchKernelGGL((k_stft_slide<N, S, FM>), dim3((unsigned)((n_strips + 256 / (N / 32) - 1) / (256 / (N / 32)))), \
                       block, 0, st, samples, frame_pfx, strip_pfx, n_tracks, n_strips, src_off, gain, hop, window, twp, \
                       rtp, mags, mag_row0, stride, fmax, redo)
#else
#define SDSP_SLIDE(N, S, FM)                                                                                      \
    hipLaunchKernelGGL((k_stft_slide2s<S, FM>), dim3((unsigned)((n_strips + 3) / 4)), block, 0, st, samples,         \
                       frame_pfx, strip_pfx, n_tracks, n_strips, src_off, gain, hop, window, twp, rtp, mags, mag_row0, \
                       stride, fmax, redo)
#endif
        if (nfft == 8192) {
            const dim3 g8((unsigned)n_strips);
            // SDSP_STFT8_CAP2 (experiment): 4 KB of dynamic LDS beside the 53 KB static make a
            // workgroup too large for 3 per CU, so the kernel runs 2 per CU
#ifdef SDSP_STFT8_CAP2
            const size_t dyn8 = 4096;
#else
            const size_t dyn8 = 0;
#endif
#ifdef SDSP_STFT8_W2
#define SDSP_K8 k_stft_slide8
#else
#define SDSP_K8 k_stft_slide8w3
#endif
            if (hop == 512)
                hipLaunchKernelGGL(SDSP_K8<1>, g8, block, dyn8, st, samples, frame_pfx, strip_pfx, n_tracks, n_strips,
                                   src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, redo);
            else
                hipLaunchKernelGGL(SDSP_K8<2>, g8, block, dyn8, st, samples, frame_pfx, strip_pfx, n_tracks, n_strips,
                                   src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, redo);
#undef SDSP_K8
        } else if (frame_max) {
            if (hop == 256)
                SDSP_SLIDE(2048, 2, true);
            else if (hop == 512)
                SDSP_SLIDE(2048, 4, true);
            else
                SDSP_SLIDE(2048, 8, true);
        } else {
            if (hop == 256)
                SDSP_SLIDE(2048, 2, false);
            else if (hop == 512)
                SDSP_SLIDE(2048, 4, false);
            else
                SDSP_SLIDE(2048, 8, false);
        }
#undef SDSP_SLIDE
        // the redo pass: a few workgroups that read the count and exit when it is 0
        const dim3 rgrid(256);
        if (nfft == 8192)
            hipLaunchKernelGGL((k_stft_mag<8192, false>), rgrid, block, 0, st, samples, frame_pfx, n_tracks, total_frames,
                               src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax, redo);
        else if (frame_max)
            hipLaunchKernelGGL((k_stft_mag<2048, true>), rgrid, block, 0, st, samples, frame_pfx, n_tracks, total_frames,
                               src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax, redo);
        else
            hipLaunchKernelGGL((k_stft_mag<2048, false>), rgrid, block, 0, st, samples, frame_pfx, n_tracks, total_frames,
                               src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax, redo);
        return;
    }
    if (nfft == 2048) {
        const dim3 grid((unsigned)((total_frames + 3) / 4));
        if (frame_max)
            hipLaunchKernelGGL((k_stft_mag<2048, true>), grid, block, 0, st, samples, frame_pfx, n_tracks,
                               total_frames, src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax, nullptr);
        else
            hipLaunchKernelGGL((k_stft_mag<2048, false>), grid, block, 0, st, samples, frame_pfx, n_tracks,
                               total_frames, src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax, nullptr);
    } else if (nfft == 8192) {
        hipLaunchKernelGGL((k_stft_mag<8192, false>), dim3((unsigned)total_frames), block, 0, st, samples, frame_pfx,
                           n_tracks, total_frames, src_off, gain, hop, window, twp, rtp, mags, mag_row0, stride, fmax,
                           nullptr);
    }
}

}  // namespace sdsp
