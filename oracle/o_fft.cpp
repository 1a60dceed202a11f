// o_fft.cpp — FFTs and the STFT of the reference path (TEST INFRASTRUCTURE, see oracle_internal.hpp).
//
// compute_stft follows src/features/chroma/extractor.rs:301-359; the FFT arithmetic is the
// sdsp specification (include/sdsp_fft_spec.h) standing in for rustfft "6.2": its STFT section
// for the spectrogram (stft_mag), its general section for the tempogram / autocorrelation FFTs
// (fft_complex, rfft).
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>

#include "oracle_internal.hpp"

namespace orc {

static inline Cx cadd(Cx a, Cx b) { return {a.re + b.re, a.im + b.im}; }
static inline Cx csub(Cx a, Cx b) { return {a.re - b.re, a.im - b.im}; }
static inline Cx cmul(Cx w, Cx z) { return {w.re * z.re - w.im * z.im, w.re * z.im + w.im * z.re}; }

struct Tw {
    std::vector<Cx> tw;  // M-point forward twiddles
};

static const std::vector<Cx>& twiddles(size_t M) {
    static std::mutex mu;
    static std::map<size_t, std::vector<Cx>> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(M);
    if (it != cache.end()) return it->second;
    std::vector<float> t(2 * M);
    sdsp_fft_twiddles((int)M, t.data());
    std::vector<Cx> v(M);
    for (size_t j = 0; j < M; j++) v[j] = {t[2 * j], t[2 * j + 1]};
    return cache.emplace(M, std::move(v)).first->second;
}

static const std::vector<Cx>& rtwiddles(size_t N) {
    static std::mutex mu;
    static std::map<size_t, std::vector<Cx>> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(N);
    if (it != cache.end()) return it->second;
    std::vector<float> t(N + 2);
    sdsp_rfft_twiddles((int)N, t.data());
    std::vector<Cx> v(N / 2 + 1);
    for (size_t k = 0; k <= N / 2; k++) v[k] = {t[2 * k], t[2 * k + 1]};
    return cache.emplace(N, std::move(v)).first->second;
}

// Stockham radix-4 (+ one radix-2) DIF, natural order in and out (sdsp_fft_spec.h).
void fft_complex(std::vector<Cx>& x) {
    const size_t M = x.size();
    if (M <= 1) return;
    if (M & (M - 1)) throw std::runtime_error("fft size must be a power of two");
    const std::vector<Cx>& tw = twiddles(M);
    std::vector<Cx> y(M);
    Cx* src = x.data();
    Cx* dst = y.data();
    size_t n = M, s = 1;
    while (n >= 4) {
        const size_t m = n / 4;
        const size_t tstep = M / n;
        for (size_t p = 0; p < m; p++) {
            const Cx w1 = tw[1 * p * tstep];
            const Cx w2 = tw[2 * p * tstep];
            const Cx w3 = tw[3 * p * tstep];
            for (size_t q = 0; q < s; q++) {
                const Cx a = src[q + s * (p)];
                const Cx b = src[q + s * (p + m)];
                const Cx c = src[q + s * (p + 2 * m)];
                const Cx d = src[q + s * (p + 3 * m)];
                const Cx apc = cadd(a, c), amc = csub(a, c), bpd = cadd(b, d), bmd = csub(b, d);
                const Cx jbmd = {bmd.im, -bmd.re};
                dst[q + s * (4 * p + 0)] = cadd(apc, bpd);
                dst[q + s * (4 * p + 1)] = cmul(w1, cadd(amc, jbmd));
                dst[q + s * (4 * p + 2)] = cmul(w2, csub(apc, bpd));
                dst[q + s * (4 * p + 3)] = cmul(w3, csub(amc, jbmd));
            }
        }
        n = m;
        s *= 4;
        std::swap(src, dst);
    }
    if (n == 2) {
        for (size_t q = 0; q < s; q++) {
            const Cx a = src[q], b = src[q + s];
            dst[q] = cadd(a, b);
            dst[q + s] = csub(a, b);
        }
        std::swap(src, dst);
    }
    if (src != x.data()) std::memcpy(x.data(), src, M * sizeof(Cx));
}

// Real-input FFT of size n (power of two >= 2): bins 0..n/2 (sdsp_fft_spec.h).
void rfft(const float* x, size_t n, std::vector<Cx>& out) {
    const size_t M = n / 2;
    std::vector<Cx> z(M);
    for (size_t j = 0; j < M; j++) z[j] = {x[2 * j], x[2 * j + 1]};
    fft_complex(z);
    const std::vector<Cx>& rt = rtwiddles(n);
    out.resize(M + 1);
    for (size_t k = 0; k <= M; k++) {
        const Cx Zk = z[k % M];
        const Cx Zr = z[(M - k) % M];
        const Cx Zc = {Zr.re, -Zr.im};
        const Cx E = {(Zk.re + Zc.re) * 0.5f, (Zk.im + Zc.im) * 0.5f};
        const Cx D = csub(Zk, Zc);
        const Cx O = {D.im * 0.5f, -(D.re * 0.5f)};
        out[k] = cadd(E, cmul(rt[k], O));
    }
}

// ---- STFT section of sdsp_fft_spec.h (the spectrogram FFTs only) ----
static inline Cx cmulf(Cx w, Cx z) {
    return {std::fma(w.re, z.re, -(w.im * z.im)), std::fma(w.re, z.im, w.im * z.re)};
}

// Stockham radix-4 (+ one radix-2) DIF with FMA complex products; the p = 0 butterflies carry
// no products (W^0 = 1).
static void stft_fft_complex(std::vector<Cx>& x, std::vector<Cx>& y) {
    const size_t M = x.size();
    if (M <= 1) return;
    if (M & (M - 1)) throw std::runtime_error("fft size must be a power of two");
    const std::vector<Cx>& tw = twiddles(M);
    y.resize(M);
    Cx* src = x.data();
    Cx* dst = y.data();
    size_t n = M, s = 1;
    while (n >= 4) {
        const size_t m = n / 4;
        const size_t tstep = M / n;
        for (size_t p = 0; p < m; p++) {
            const Cx w1 = tw[1 * p * tstep];
            const Cx w2 = tw[2 * p * tstep];
            const Cx w3 = tw[3 * p * tstep];
            for (size_t q = 0; q < s; q++) {
                const Cx a = src[q + s * (p)];
                const Cx b = src[q + s * (p + m)];
                const Cx c = src[q + s * (p + 2 * m)];
                const Cx d = src[q + s * (p + 3 * m)];
                const Cx apc = cadd(a, c), amc = csub(a, c), bpd = cadd(b, d), bmd = csub(b, d);
                const Cx t1 = {amc.re + bmd.im, amc.im - bmd.re};  // amc + (-i)(b - d)
                const Cx t2 = csub(apc, bpd);
                const Cx t3 = {amc.re - bmd.im, amc.im + bmd.re};  // amc - (-i)(b - d)
                dst[q + s * (4 * p + 0)] = cadd(apc, bpd);
                dst[q + s * (4 * p + 1)] = p ? cmulf(w1, t1) : t1;
                dst[q + s * (4 * p + 2)] = p ? cmulf(w2, t2) : t2;
                dst[q + s * (4 * p + 3)] = p ? cmulf(w3, t3) : t3;
            }
        }
        n = m;
        s *= 4;
        std::swap(src, dst);
    }
    if (n == 2) {
        for (size_t q = 0; q < s; q++) {
            const Cx a = src[q], b = src[q + s];
            dst[q] = cadd(a, b);
            dst[q + s] = csub(a, b);
        }
        std::swap(src, dst);
    }
    if (src != x.data()) std::memcpy(x.data(), src, M * sizeof(Cx));
}

// |X[k]|, k = 0..n/2, of a real frame of n samples: z[j] = (x[2j], x[2j+1]), Z = FFT_M(z),
// S = Z[k] + conj(Z[M-k]), D' = -i (Z[k] - conj(Z[M-k])), Y = S + rt[k] D' (two FMAs per
// component), |X[k]| = 2^-33 * sqrt(fma(Y.re, Y.re, Y.im * Y.im)) (the frame carries the window's
// 2^32, so Y = 2^33 X); the post twiddles are symmetric,
// rt[M-k] = (-rt[k].re, rt[k].im) for 0 <= k < M/2.
// `post` is 2^-33 for the scaled evaluation and 1 for the overflow rule's (compute_stft); the
// return value tells whether some fma(Y.re, Y.re, Y.im * Y.im) overflowed to +inf.
static bool stft_mag(const float* x, size_t n, float* mag, std::vector<Cx>& z, std::vector<Cx>& tmp,
                     float post = 0x1p-33f) {
    const size_t M = n / 2;
    z.resize(M);
    for (size_t j = 0; j < M; j++) z[j] = {x[2 * j], x[2 * j + 1]};
    stft_fft_complex(z, tmp);
    const std::vector<Cx>& rt = rtwiddles(n);
    bool ovf = false;
    for (size_t k = 0; k <= M; k++) {
        const Cx Zk = z[k % M];
        const Cx Zr = z[(M - k) % M];
        // symmetric post twiddles: rt[k] for k <= M/2, rt[M-k] := (-rt[k].re, rt[k].im) for k > M/2
        const Cx w = k > M / 2 ? Cx{-rt[M - k].re, rt[M - k].im} : rt[k];
        const float sre = Zk.re + Zr.re, sim = Zk.im - Zr.im;
        const float dre = Zk.im + Zr.im, dim = -(Zk.re - Zr.re);
        const float yre = std::fma(w.re, dre, std::fma(-w.im, dim, sre));
        const float yim = std::fma(w.re, dim, std::fma(w.im, dre, sim));
        const float e = std::fma(yre, yre, yim * yim);
        ovf |= e == INFINITY;
        mag[k] = post * std::sqrt(e);
    }
    return ovf;
}

// extractor.rs:301-359
Spec compute_stft(const float* s, size_t n_samples, size_t frame_size, size_t hop) {
    Spec out;
    if (n_samples < frame_size) return out;  // :310-313
    const size_t n_frames = (n_samples - frame_size) / hop + 1;
    const size_t n_bins = frame_size / 2 + 1;
    std::vector<float> window(frame_size);
    // the STFT section's window carries 2^32 (exact; |X| carries 2^-33, see stft_mag)
    for (size_t i = 0; i < frame_size; i++) window[i] = sdsp_hann_f32((int)i, (int)frame_size) * 0x1p32f;
    out.frames = n_frames;
    out.bins = n_bins;
    out.d.resize(n_frames * n_bins);
    std::vector<float> buf(frame_size);
    std::vector<Cx> z, tmp;
    for (size_t f = 0; f < n_frames; f++) {
        const float* fr = s + f * hop;
        for (size_t i = 0; i < frame_size; i++) buf[i] = fr[i] * window[i];
        if (stft_mag(buf.data(), frame_size, out.row(f), z, tmp)) {
            // the overflow rule (sdsp_fft_spec.h STFT section): some |Y|^2 = 2^66 |X|^2 overflowed,
            // so the frame is evaluated again in the reference's own range, Y = X
            // (extractor.rs:352 overflows only where (re*re + im*im) itself does)
            for (size_t i = 0; i < frame_size; i++) buf[i] = (fr[i] * window[i]) * 0x1p-33f;
            stft_mag(buf.data(), frame_size, out.row(f), z, tmp, 1.0f);
        }
    }
    return out;
}

}  // namespace orc
