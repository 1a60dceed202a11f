/*
 * sdsp_fft_spec.h — the arithmetic specification of every FFT on the analyze_audio path.
 *
 * The reference computes all FFTs with rustfft "6.2" (Cargo.toml:18; call sites
 * src/features/chroma/extractor.rs:326-346, src/features/period/tempogram_fft.rs:149-151,
 * src/features/period/autocorrelation.rs:240-251).  rustfft's planner picks an
 * implementation-defined algorithm and SIMD path, so the reference does not pin the
 * rounding of its FFT outputs ("parity unpinned").  sdsp pins it:
 *
 *   complex FFT, size M = 2^m, forward (e^{-2 pi i jk/M}), no scaling:
 *     Stockham autosort, decimation in frequency, radix-4 stages while the current
 *     sub-transform length n >= 4, then one radix-2 stage if n == 2.  One radix-4 stage
 *     with stride s (s = 1, 4, 16, ...) and m = n/4, for p < m, q < s:
 *        a = x[q + s(p)],  b = x[q + s(p+m)],  c = x[q + s(p+2m)],  d = x[q + s(p+3m)]
 *        apc = a + c;  amc = a - c;  bpd = b + d;  bmd = b - d
 *        jbmd = (bmd.im, -bmd.re)                     (-i * (b - d))
 *        y[q + s(4p+0)] = apc + bpd
 *        y[q + s(4p+1)] = W^{1p} * (amc + jbmd)
 *        y[q + s(4p+2)] = W^{2p} * (apc - bpd)
 *        y[q + s(4p+3)] = W^{3p} * (amc - jbmd)
 *     with W^{kp} = tw[k*p*(M/n)] from the M-point table below, and the complex product
 *        (w * z) = (w.re*z.re - w.im*z.im,  w.re*z.im + w.im*z.re)   (two roundings each,
 *        no FMA).  Radix-2 stage (n == 2): y[q] = x[q] + x[q+s]; y[q+s] = x[q] - x[q+s].
 *
 *   real-input FFT of size N = 2M: z[j] = (x[2j], x[2j+1]); Z = FFT_M(z); for k = 0..M:
 *        Zk = Z[k mod M]; Zc = conj(Z[(M-k) mod M])
 *        E = ((Zk.re + Zc.re)*0.5, (Zk.im + Zc.im)*0.5)
 *        D = Zk - Zc;  O = (D.im*0.5, -(D.re*0.5))
 *        X[k] = E + rt[k] * O,  rt[k] = e^{-2 pi i k/N}
 *     |X[k]| = sqrt(X.re*X.re + X.im*X.im);  power = X.re*X.re + X.im*X.im.
 *
 * STFT section (round 2; the spectrogram FFTs of compute_stft only -- the tempogram and
 * autocorrelation FFTs keep the general section above).  Same Stockham radix-4 (+ radix-2)
 * stages and tables, with
 *   - complex products in FMA form: (w * z) = (fma(w.re, z.re, -(w.im*z.im)),
 *                                             fma(w.re, z.im, w.im*z.re));
 *   - no products for the p = 0 butterflies (W^0 = 1): y1 = amc + jbmd, y2 = apc - bpd,
 *     y3 = amc - jbmd;
 *   - post twiddles symmetric about M/2: rt[k] from the table for k <= M/2, and
 *     rt[M-k] := (-rt[k].re, rt[k].im) for 0 <= k < M/2 (e^{-i(pi - t)} = -conj(e^{-it}));
 *   - post-processing for k = 0..M, with Zk = Z[k mod M], Zr = Z[(M-k) mod M]:
 *        S = (Zk.re + Zr.re, Zk.im - Zr.im)              (Zk + conj(Zr))
 *        D' = (Zk.im + Zr.im, -(Zk.re - Zr.re))          (-i (Zk - conj(Zr)))
 *        Y.re = fma(rt.re, D'.re, fma(-rt.im, D'.im, S.re))
 *        Y.im = fma(rt.re, D'.im, fma(rt.im, D'.re, S.im))
 *        |X[k]| = 2^-33 * sqrt(fma(Y.re, Y.re, Y.im * Y.im))    (sqrt correctly rounded)
 *     where the frame is windowed with w[i] * 2^32 (an exact scaling of the Hann table), so
 *     Y = 2^33 X: |X|^2 * 2^66 stays above the subnormal range for any audible input, the range in
 *     which the kernels' fast correctly rounded sqrt is exact, and the scaling itself changes no
 *     rounding (powers of two commute with round-to-nearest away from subnormals);
 *   - overflow rule: if some fma(Y.re, Y.re, Y.im * Y.im) of a frame is +inf (|X| >= 2^31, e.g.
 *     unnormalised int-scale PCM), the whole frame is evaluated again with the windowed samples
 *     times 2^-33 (so Y = X, the reference's own range: extractor.rs:352 overflows only where
 *     re*re + im*im does) and |X[k]| = sqrt(fma(Y.re, Y.re, Y.im * Y.im));
 * FMA is a single rounding on both sides (gfx950 v_fma_f32 / x86 vfmadd), so the STFT stays
 * bit-identical between the CPU restatement and the kernels, at about two thirds of the
 * general section's arithmetic.  tests/test_spec.py checks it against numpy float64 too.
 *
 * Twiddles are cos/sin evaluated in double by sdsp_libm and rounded once to f32.  Both the
 * CPU restatement (oracle/) and the HIP kernels implement exactly this operation order, so
 * their spectra agree bit for bit; tests/test_spec.py checks the specification
 * against numpy's float64 FFT (relative error <= 2e-6 of the frame's peak).
 */
#ifndef SDSP_FFT_SPEC_H
#define SDSP_FFT_SPEC_H

#include "sdsp_libm.h"

#define SD_TWO_PI_D 6.28318530717958647692e+00
#define SD_PIO2_D 1.57079632679489661923e+00

/* tw[j] = e^{-2 pi i j / M}, j = 0..M-1, as interleaved (re, im) f32 pairs */
static inline void sdsp_fft_twiddles(int M, float* tw_interleaved) {
    for (int j = 0; j < M; j++) {
        double th = SD_TWO_PI_D * (double)j / (double)M;
        double c = sd_cos_d(th);
        double s = sd_cos_d(th - SD_PIO2_D); /* sin(th) */
        tw_interleaved[2 * j] = (float)c;
        tw_interleaved[2 * j + 1] = (float)(-s);
    }
}

/* rt[k] = e^{-2 pi i k / N}, k = 0..N/2, as interleaved (re, im) f32 pairs */
static inline void sdsp_rfft_twiddles(int N, float* rt_interleaved) {
    for (int k = 0; k <= N / 2; k++) {
        double th = SD_TWO_PI_D * (double)k / (double)N;
        double c = sd_cos_d(th);
        double s = sd_cos_d(th - SD_PIO2_D);
        rt_interleaved[2 * k] = (float)c;
        rt_interleaved[2 * k + 1] = (float)(-s);
    }
}

/*
 * Symmetric Hann window exactly as extractor.rs:318-323 / tempogram_fft.rs:122-128:
 *   x = 2.0 * PI * i as f32 / (n - 1) as f32;  w = 0.5 * (1.0 - x.cos())
 * (all f32 operations, left to right).
 */
SD_HD float sdsp_hann_f32(int i, int n) {
    const float PI_F = 3.14159265358979323846f;
    float x = 2.0f * PI_F * (float)i / (float)(n - 1);
    return 0.5f * (1.0f - sd_cosf(x));
}

#endif /* SDSP_FFT_SPEC_H */
