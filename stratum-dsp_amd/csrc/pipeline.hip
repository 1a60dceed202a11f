// pipeline.hip — analyze_audio() for a batch of tracks on one MI355X (reference src/lib.rs:86-1635),
// plus the C ABI entry points (sdsp_analyze_audio / _batch / _batch_device, synthetic tracks).
//
// Per sub-batch (sized to an HBM budget), the host plans ragged per-track frame ranges and
// launches:
//   A  peak/gain, silence RMS, trim                      -> host reads trim bounds (sync 1)
//   E  key, forked onto the key stream: STFT 8192/512 (key_stft_frame_size / hop; the tempo
//      path's frame_size / hop_size without the override) -> harmonic mask (in place) -> HPCP ->
//      key vote (runs under B-D)
//   B  energy RMS + energy-flux onsets; STFT 2048/512 (frame_size / hop_size); frame features;
//      spectral/HFC onsets;
//      consensus; novelty (5 variants); FFT + ACF tempograms; candidate scoring + gate
//                                                        -> host reads estimates (sync 2)
//   C  escalation for ambiguous tracks: STFT 2048/256 and 2048/1024 of those tracks, the same
//      feature/novelty/tempogram/scoring kernels, then multi-resolution fusion
//   D  beat grid; join the key stream                    -> host reads results (sync 3)
// No stage falls back to the CPU; host code only plans offsets and formats the result.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sdsp_fft_spec.h"
#include "batch_sched.hpp"
#include "kernels.hpp"
#include "sdsp_runtime.hpp"

namespace sdsp {

namespace {

// Spectrogram row strides (floats; multiples of 4 for 16-B rows).  The key spectrogram's rows
// are 16 KiB + 256 B apart: at 16 KiB + 16 B the mask's column streams (one 256-B row segment
// per wave per frame) run 1.5x slower (profiles/README.md, stride sweep of round 2).
constexpr int STRIDE2 = 1028;  // 1025 bins
constexpr int STRIDE8 = 4160;  // 4097 bins
// row stride of the tempo path's spectrogram for AnalysisConfig::frame_size (nb = fs/2 + 1 bins)
static int base_stride(int fs) {
    if (fs == 2048) return STRIDE2;
    if (fs == 8192) return STRIDE8;
    return (fs / 2 + 1 + 3) & ~3;
}
// the key spectrogram's frame size and hop (src/lib.rs:985-1009): the override's, else the tempo
// path's frame_size / hop_size (whose spectrogram the reference reuses; the engine recomputes it
// on the key stream, bit-identical by the STFT spec)
static uint64_t key_fft(const sdsp_config& c) {
    return c.enable_key_stft_override ? std::max<uint64_t>(c.key_stft_frame_size, 256) : c.frame_size;
}
static uint64_t key_hop(const sdsp_config& c) {
    return c.enable_key_stft_override ? std::max<uint64_t>(c.key_stft_hop_size, 1) : c.hop_size;
}
constexpr int SUPPORT_HMAX = 8;

uint64_t next_pow2(uint64_t n) {
    uint64_t p = 1;
    while (p < n) p <<= 1;
    return p;
}

// ---------------------------------------------------------------------------------------
// Host-side constant tables (identical arithmetic to the reference; sdsp_libm on both sides)
struct MelTable {
    std::vector<int> m;    // 2 per bin, -1 = none
    std::vector<float> w;  // 2 per bin
    int n_mels = 0;
};

// MelFilterbank::new, novelty.rs:83-165
MelTable mel_table(uint32_t sr, int n_bins, int n_mels_in, float fmin_hz, float fmax_hz, std::string* err) {
    MelTable t;
    const int n_mels = std::max(n_mels_in, 4);
    t.n_mels = n_mels;
    const float nyq = (float)sr * 0.5f;
    const float fmin = sd_minf(sd_maxf(fmin_hz, 0.0f), sd_maxf(nyq, 1.0f));
    float fmax = fmax_hz;
    if (!(sd_isfinite_f(fmax) && fmax > 0.0f)) fmax = nyq;
    fmax = sd_clampf(fmax, fmin + 1.0f, nyq);
    const int fft_size = (n_bins - 1) * 2;
    const float fres = (float)sr / (float)fft_size;
    auto mel = [](float f) { return 2595.0f * sd_log10f(1.0f + (f / 700.0f)); };
    auto inv_mel = [](float v) { return 700.0f * (sd_powf(10.0f, v / 2595.0f) - 1.0f); };
    const float mmin = mel(fmin), mmax = mel(fmax);
    const float step = (mmax - mmin) / (float)(n_mels + 1);
    std::vector<int> bp((size_t)n_mels + 2);
    for (int i = 0; i < n_mels + 2; i++) {
        const float hz = inv_mel(mmin + step * (float)i);
        int64_t b = sd_f2i64(sd_roundf(hz / fres));
        b = std::max<int64_t>(0, std::min<int64_t>(b, n_bins - 1));
        bp[(size_t)i] = (int)b;
    }
    for (size_t i = 1; i < bp.size(); i++)
        if (bp[i] <= bp[i - 1]) bp[i] = std::min(bp[i - 1] + 1, n_bins - 1);
    t.m.assign((size_t)n_bins * 2, -1);
    t.w.assign((size_t)n_bins * 2, 0.0f);
    std::vector<int> cnt((size_t)n_bins, 0);
    auto push = [&](int b, int m, float w) {
        if (cnt[(size_t)b] >= 2) {
            *err = "mel filterbank: more than two contributions for one bin";
            return;
        }
        t.m[(size_t)b * 2 + cnt[(size_t)b]] = m;
        t.w[(size_t)b * 2 + cnt[(size_t)b]] = w;
        cnt[(size_t)b]++;
    };
    for (int mm = 0; mm < n_mels; mm++) {
        const int l = bp[(size_t)mm], c = bp[(size_t)mm + 1], r = bp[(size_t)mm + 2];
        if (!(l < c && c < r)) continue;
        for (int b = l; b <= c; b++) {
            const float w = b == l ? 0.0f : ((float)b - (float)l) / ((float)c - (float)l);
            if (w > 0.0f) push(b, mm, w);
        }
        for (int b = c; b <= r; b++) {
            const float w = b == r ? 0.0f : ((float)r - (float)b) / ((float)r - (float)c);
            if (w > 0.0f) push(b, mm, w);
        }
    }
    return t;
}

// Register-pair schedule for the mel sums (see k_features.hip): mels are flushed in index
// order; every contribution of a bin must land on the two live accumulators mA, mA+1.
std::vector<MelPlan> mel_plan(const MelTable& t, int n_bins, std::string* err) {
    std::vector<MelPlan> p((size_t)n_bins, MelPlan{0, 0, 0, 0.0f, 0.0f});
    int mA = 0;
    for (int b = 0; b < n_bins; b++) {
        int mx = -1;
        for (int s = 0; s < 2; s++) mx = std::max(mx, t.m[(size_t)b * 2 + s]);
        if (mx < 0) continue;
        const int nf = std::max(0, mx - (mA + 1));
        MelPlan& q = p[(size_t)b];
        q.nflush = nf;
        mA += nf;
        for (int s = 0; s < 2; s++) {
            const int m = t.m[(size_t)b * 2 + s];
            if (m < 0) continue;
            if (m != mA && m != mA + 1) *err = "mel filterbank: contributions not on adjacent mels";
            (s == 0 ? q.s0 : q.s1) = m - mA;
            (s == 0 ? q.w0 : q.w1) = t.w[(size_t)b * 2 + s];
        }
    }
    return p;
}

// hz_to_bin, tempogram.rs:279-289
int hz_to_bin(float f, float fres, int n_bins) {
    if (!sd_isfinite_f(f) || f <= 0.0f || !sd_isfinite_f(fres) || fres <= 0.0f) return 0;
    int64_t b = sd_f2i64(sd_roundf(f / fres));
    return (int)std::max<int64_t>(0, std::min<int64_t>(b, (int64_t)n_bins - 1));
}

// compiler-rt __powisf2 (Rust f32::powi)
float powi_f(float a, int b) {
    const bool recip = b < 0;
    float r = 1.0f;
    while (true) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1.0f / r : r;
}

// per-(bin, harmonic) HPCP decisions, extractor.rs:636-668 (tuning 0)
std::vector<HarmEntry> harm_table(int B, uint32_t sr, int fft_size, float sigma_in, int hmax, float decay_in) {
    std::vector<HarmEntry> t((size_t)B * HP_HMAX);
    const float fres = (float)sr / (float)fft_size;
    const float fmin = sd_maxf(100.0f, 20.0f), fmax = sd_minf(5000.0f, (float)sr / 2.0f);
    const float sigma = sd_maxf(sigma_in, 1e-6f);
    const float decay = sd_clampf(decay_in, 0.0f, 1.0f);
    for (int bin = 0; bin < B; bin++) {
        const float f0 = (float)bin * fres;
        for (int h = 1; h <= HP_HMAX; h++) {
            HarmEntry& e = t[(size_t)bin * HP_HMAX + (size_t)(h - 1)];
            e = HarmEntry{};
            const float fh = f0 * (float)h;
            if (h > hmax || fh > fmax) {
                e.state = 0;
                continue;
            }
            if (fh < fmin) {
                e.state = 1;
                continue;
            }
            e.state = 2;
            const float semitone = 12.0f * sd_log2f(fh / 440.0f) + 57.0f - 0.0f;
            const float spc = sd_rem_euclid_f(semitone, 12.0f);
            const float ppc = sd_rem_euclid_f(sd_roundf(spc), 12.0f);
            const int primary = sd_f2i32(ppc);
            e.hw = powi_f(decay, h - 1) / (float)h;
            for (int o = -1; o <= 1; o++) {
                const int tc = (((primary + o) % 12) + 12) % 12;
                float dist = sd_absf(spc - (float)tc);
                dist = sd_minf(dist, 12.0f - dist);
                e.tc[o + 1] = tc;
                e.wt[o + 1] = sd_expf(-dist * dist / (2.0f * sigma * sigma));
            }
        }
    }
    return t;
}

// Contiguous candidate bins of a band, as the reference's peak loops visit them:
// `for bin in 1..len-1 { if f < fmin continue; if f > fmax break; ... }` (extractor.rs:599-617).
// Leaves *lo > *hi when the band is empty.
void band_bins(int B, float fres, float fmin, float fmax, int* lo, int* hi) {
    *lo = 1;
    *hi = 0;
    if (!(fmax > fmin)) return;
    int l = -1, h = -1;
    for (int b = 1; b + 1 < B; b++) {
        const float f = (float)b * fres;
        if (f < fmin) continue;
        if (f > fmax) break;
        if (l < 0) l = b;
        h = b;
    }
    if (l >= 0) *lo = l, *hi = h;
}

// HPCP's peak band of the key spectrogram (bins pk_lo .. pk_hi; empty when lo > hi), and whether a
// configuration takes the default key path's band-limited mask with block-folded frame energies
// (k_mask_rp / k_hpcp_band): the harmonic mask at margin 12 and power 2, plain HPCP,
// nothing else reading the masked spectrogram.  SDSP_KEY_EXACT_ENERGY builds never take it.
void key_peak_band(const sdsp_config& c, uint32_t sr, int* lo, int* hi) {
    const int kfs = (int)std::min<uint64_t>(key_fft(c), STFT_GEN_MAX);
    band_bins(kfs / 2 + 1, (float)sr / (float)kfs, sd_maxf(100.0f, 20.0f), sd_minf(5000.0f, (float)sr / 2.0f), lo, hi);
}
bool key_energy_blocked(const sdsp_config& c, uint32_t sr) {
#ifdef SDSP_KEY_EXACT_ENERGY
    return false;
#else
    const bool use_log = c.enable_key_log_frequency;
    const bool tuned = c.enable_key_tuning_compensation && !use_log;
    const bool whiten = c.enable_key_hpcp_whitening && c.key_hpcp_whitening_smooth_bins >= 3;
    const bool plain_hpcp = !use_log && c.enable_key_hpcp && !tuned && !whiten && !c.enable_key_hpcp_bass_blend;
    int lo = 1, hi = 0;
    key_peak_band(c, sr, &lo, &hi);
    // the scoring whose energy-dependent decisions k_key_vote certifies (KeyParams::near_check):
    // segment voting or the full slice, without the mode heuristic, ensemble or multi-scale voting
    const bool plain_scoring = !c.enable_key_mode_heuristic && !c.enable_key_minor_harmonic_bonus &&
                               !c.enable_key_ensemble && !(c.enable_key_multi_scale && c.key_multi_scale_lengths_len > 0);
    return plain_hpcp && plain_scoring && !c.enable_key_hpss_harmonic && c.enable_key_harmonic_mask &&
           mask_band_ok((int)c.key_spectrogram_smooth_margin, c.key_harmonic_mask_power) &&
           !(c.enable_key_beat_synchronous && !c.enable_key_log_frequency) && lo <= hi;
#endif
}

// estimate_tuning_offset_semitones_from_spectrogram over [80, 2000] Hz (src/lib.rs:1101-1109,
// extractor.rs:98-140): the band is every bin with fmin <= f <= fmax
TuningParams tuning_params(const sdsp_config& c, uint32_t sr, int B, float fres, int stride) {
    TuningParams t{};
    t.stride = stride;
    const float fmin = sd_maxf(80.0f, 20.0f);
    const float fmax = sd_clampf(2000.0f, fmin + 1.0f, (float)sr / 2.0f);
    t.lo = 1;
    t.hi = 0;
    for (int b = 0; b < B; b++) {
        const float f = (float)b * fres;
        if (f < fmin) continue;
        if (f > fmax) break;
        if (t.lo > t.hi) t.lo = b;
        t.hi = b;
    }
    t.step = (int)std::min<uint64_t>(std::max<uint64_t>(c.key_tuning_frame_step, 1), INT32_MAX);
    const int tb = t.hi - t.lo + 1;
    t.chf = tb > 0 ? std::max(1, std::min(8, 4096 / tb)) : 1;
    t.fres = fres;
    t.thr = sd_clampf(c.key_tuning_peak_rel_threshold, 0.0f, 1.0f);
    t.lim = sd_absf(c.key_tuning_max_abs_semitones);
    return t;
}

// k_chroma parameters: mode 0 frame_to_chroma_tuned (extractor.rs:393-481), mode 1 the
// log-frequency conversion (extractor.rs:701-828, fmin 100, fmax 5000 from src/lib.rs:1068-1073)
ChromaParams chroma_params(const sdsp_config& c, uint32_t sr, int mode, int B, float fres, int stride) {
    ChromaParams p{};
    p.B = B;
    p.stride = stride;
    p.fres = fres;
    p.soft = c.soft_chroma_mapping ? 1 : 0;
    p.sigma = c.soft_mapping_sigma;
    p.gate_small = 1;
    p.lo = 1;
    p.hi = 0;
    const float nyq = (float)sr / 2.0f;
    if (mode == 0) {
        const float top = sd_minf(5000.0f, nyq);
        for (int b = 0; b < B; b++) {
            const float f = (float)b * fres;
            if (f < 100.0f) continue;
            if (f > top || f >= nyq) break;
            if (p.lo > p.hi) p.lo = b;
            p.hi = b;
        }
    } else {
        const float fmin = sd_maxf(100.0f, 20.0f), fmax = sd_minf(5000.0f, nyq - 1.0f);
        const float smin = 12.0f * sd_log2f(fmin / 440.0f) + 57.0f;
        const float smax = 12.0f * sd_log2f(fmax / 440.0f) + 57.0f;
        p.bmin = sd_f2i32(__builtin_floorf(smin));
        p.n_log = sd_f2i32(__builtin_ceilf(smax)) - p.bmin + 1;
        p.log_off = sd_f2i32(__builtin_floorf(12.0f * sd_log2f(100.0f / 440.0f) + 57.0f));
        for (int b = 0; b < B; b++) {
            const float f = (float)b * fres;
            if (f < fmin || f >= fmax || f >= nyq) continue;
            if (p.lo > p.hi) p.lo = b;
            p.hi = b;
        }
    }
    return p;
}

// k_hpcp_x parameters (extractor.rs:529-680 with whitening, :1154-1244 bass blend)
HpcpXParams hpcp_x_params(const sdsp_config& c, uint32_t sr, int B, float fres, bool whiten, int stride) {
    HpcpXParams h{};
    h.B = B;
    h.stride = stride;
    h.fres = fres;
    h.fmin = sd_maxf(100.0f, 20.0f);
    h.fmax = sd_minf(5000.0f, (float)sr / 2.0f);
    h.main_ok = h.fmax > h.fmin;
    band_bins(B, fres, h.fmin, h.fmax, &h.pk_lo, &h.pk_hi);
    h.K = (int)std::max<uint64_t>(c.key_hpcp_peaks_per_frame, 1);
    h.hmax = (int)std::max<uint64_t>(c.key_hpcp_num_harmonics, 1);
    h.p = sd_clampf(c.key_hpcp_mag_power, 0.05f, 1.0f);
    h.decay = sd_clampf(c.key_hpcp_harmonic_decay, 0.0f, 1.0f);
    h.sigma = c.soft_mapping_sigma;
    h.bass = c.enable_key_hpcp_bass_blend ? 1 : 0;
    h.bk_lo = 1;
    h.bk_hi = 0;
    if (h.bass) {
        h.bfmin = sd_maxf(c.key_hpcp_bass_fmin_hz, 20.0f);
        h.bfmax = sd_minf(c.key_hpcp_bass_fmax_hz, (float)sr / 2.0f);
        h.bass_ok = h.bfmax > h.bfmin;
        band_bins(B, fres, h.bfmin, h.bfmax, &h.bk_lo, &h.bk_hi);
        h.KB = (int)std::min<uint64_t>(std::max<uint64_t>(c.key_hpcp_peaks_per_frame, 1), 12);
        h.bw = sd_clampf(c.key_hpcp_bass_weight, 0.0f, 1.0f);
    }
    if (whiten) {
        const int win = (int)(std::max<uint64_t>(c.key_hpcp_whitening_smooth_bins, 3) | 1);
        h.half = win / 2;
        int rp = 1, rx = 1;
        while (rp < 2 * h.half + 2) rp <<= 1;
        while (rx < h.half + 1) rx <<= 1;
        h.rp = rp, h.rp_mask = rp - 1, h.rx = rx, h.rx_mask = rx - 1;
    }
    return h;
}

// harmonic_spectrogram_hpss_median_mask's band and windows (extractor.rs:1400-1420, with
// fmin 100 / fmax 5000 from src/lib.rs:1014-1024); nb = 0 when the band is empty
KeyHpssParams key_hpss_params(const sdsp_config& c, uint32_t sr, int B, float fres, int stride) {
    KeyHpssParams k{};
    k.B = B;
    k.stride = stride;
    const float fmin = sd_maxf(100.0f, 20.0f);
    const float fmax = sd_clampf(5000.0f, fmin + 1.0f, (float)sr / 2.0f);
    int64_t bs = sd_f2i64(__builtin_floorf(fmin / fres)), be = sd_f2i64(__builtin_ceilf(fmax / fres));
    bs = std::min<int64_t>(std::max<int64_t>(bs, 0), B);
    be = std::min<int64_t>(std::max<int64_t>(be, 0), B);
    k.bin0 = (int)bs;
    k.nb = be > bs ? (int)(be - bs) : 0;
    k.step = (int)std::min<uint64_t>(std::max<uint64_t>(c.key_hpss_frame_step, 1), INT32_MAX);
    k.tm = (int)std::min<uint64_t>(c.key_hpss_time_margin, 1u << 20);
    k.fm = (int)std::min<uint64_t>(c.key_hpss_freq_margin, 1u << 20);
    k.p = sd_maxf(c.key_hpss_mask_power, 1.0f);
    return k;
}

// Configuration support that depends on the sample rate.
std::string unsupported_sr(const sdsp_config& c, uint32_t sr) {
    if (sr == 0) return "";
    const int kfs = (int)std::min<uint64_t>(key_fft(c), STFT_GEN_MAX);
    const int B8 = kfs / 2 + 1, ks = base_stride(kfs);
    const float fres = (float)sr / (float)kfs;
    if (c.enable_key_log_frequency) {
        const ChromaParams p = chroma_params(c, sr, 1, B8, fres, ks);
        if (p.n_log <= 0) return "degenerate key log-frequency range (sample rate too low)";
        if ((size_t)(p.hi - p.lo + 1) * sizeof(ChromaBin) > 65536) return "log-frequency chroma band > 3276 bins";
    } else if (c.enable_key_tuning_compensation) {
        const TuningParams t = tuning_params(c, sr, B8, fres, ks);
        if (t.hi - t.lo + 1 > 4096) return "tuning band > 4096 bins";
    }
    if (!c.enable_key_log_frequency && !c.enable_key_hpcp) {
        const ChromaParams p = chroma_params(c, sr, 0, B8, fres, ks);
        if ((size_t)(p.hi - p.lo + 1) * sizeof(ChromaBin) > 65536) return "chroma band > 3276 bins (sample rate too low)";
    }
    return "";
}

// templates.rs:64-145 (Krumhansl-Kessler) and :147-235 (Temperley): rows 0-23 K-K major/minor
// keys, rows 24-47 Temperley; each profile rotated to the key, then L2-normalised.
void key_templates(float* out /*48x12*/) {
    const float kM[12] = {6.35f, 2.23f, 3.48f, 2.33f, 4.38f, 4.09f, 2.52f, 5.19f, 2.39f, 3.66f, 2.29f, 2.88f};
    const float km[12] = {6.33f, 2.68f, 3.52f, 5.38f, 2.60f, 3.53f, 2.54f, 4.75f, 3.98f, 2.69f, 3.34f, 3.17f};
    const float tM[12] = {5.0f, 2.0f, 3.5f, 2.0f, 4.5f, 4.0f, 2.0f, 4.5f, 2.0f, 3.5f, 1.5f, 4.0f};
    const float tm[12] = {5.0f, 2.0f, 3.5f, 5.0f, 2.0f, 3.5f, 2.0f, 4.5f, 3.5f, 2.0f, 4.0f, 3.5f};
    for (int k = 0; k < 48; k++) {
        float* v = out + k * 12;
        const float* base = k < 24 ? (k < 12 ? kM : km) : (k < 36 ? tM : tm);
        const int key = k % 12;
        for (int s = 0; s < 12; s++) v[s] = base[(s + 12 - key) % 12];
        float sq = 0.0f;
        for (int i = 0; i < 12; i++) sq += v[i] * v[i];
        const float n = __builtin_sqrtf(sq);
        if (n > 1e-12f)
            for (int i = 0; i < 12; i++) v[i] /= n;
    }
}

// RMS / LUFS constants (normalization.rs:119-158, 183-259, 325-470; lib.rs:118-122 fixes
// target_loudness_lufs = -14 and max_headroom_db = 1).  The K-weighting coefficients use the C
// library's sinf/cosf, the functions f32::sin/cos lower to.
LoudnessParams loudness_params(int method, uint32_t sr) {
    LoudnessParams p{};
    p.method = method == SDSP_NORM_RMS ? 1 : 2;
    const float target_lufs = -14.0f, headroom = 1.0f;
    p.target_lufs = target_lufs;
    p.target_rms = sd_powf(10.0f, ((target_lufs + 3.0f) - headroom) / 20.0f);
    p.target_peak = sd_powf(10.0f, (0.0f - headroom) / 20.0f);
    p.gate = sd_powf(10.0f, (-70.0f + 0.691f) / 10.0f);
    const float fsr = (float)sr;
    p.block = (int64_t)sd_f2u64(fsr * 400.0f / 1000.0f);
    const float w0 = 2.0f * 3.14159274f * 1681.9745f / fsr;
    const float cw = cosf(w0), sw = sinf(w0);
    const float alpha = sw / 2.0f * sqrtf(1.0f / 0.707f);
    const float b0 = (1.0f + cw) / 2.0f, b1 = -(1.0f + cw), b2 = (1.0f + cw) / 2.0f;
    const float a0 = 1.0f + alpha, a1 = -2.0f * cw, a2 = 1.0f - alpha;
    p.b0 = b0 / a0;
    p.b1 = b1 / a0;
    p.b2 = b2 / a0;
    p.a1 = a1 / a0;
    p.a2 = a2 / a0;
    return p;
}

// autocorrelation_tempogram's BPM grid and lags for one hop (tempogram_autocorr.rs:128-140)
void acf_grid(uint32_t sr, int hop, float min_bpm, float max_bpm, float res, std::vector<float>* bpms,
              std::vector<int>* lags) {
    const float frame_rate = (float)sr / (float)hop;
    for (float bpm = min_bpm; bpm <= max_bpm; bpm += res) {
        const float bps = bpm / 60.0f;
        const float fpb = frame_rate / bps;
        bpms->push_back(bpm);
        lags->push_back((int)std::min<uint64_t>(sd_f2u64(fpb), (uint64_t)INT32_MAX));
    }
}

// in-range FFT-tempogram bins for size P (tempogram_fft.rs:158-175)
void fft_bins(uint32_t sr, int hop, uint64_t P, float min_bpm, float max_bpm, int* b_lo, int* K, float* fres_out) {
    const float frame_rate = (float)sr / (float)hop;
    const float fres = frame_rate / (float)P;
    *fres_out = fres;
    int lo = -1, hi = -2;
    for (uint64_t b = 0; b <= P / 2; b++) {
        const float bpm = (float)b * fres * 60.0f;
        if (bpm >= min_bpm && bpm <= max_bpm) {
            if (lo < 0) lo = (int)b;
            hi = (int)b;
        }
    }
    *b_lo = lo < 0 ? 0 : lo;
    *K = lo < 0 ? 0 : hi - lo + 1;
}

std::string fmt2(float v) {
    char b[64];
    std::snprintf(b, sizeof b, "%.2f", (double)v);
    return b;
}

// ---------------------------------------------------------------------------------------
struct Ctx {
    DeviceCtx& d;
    std::deque<std::vector<uint8_t>> keep;  // host staging kept alive until the next sync
    std::string pre;  // buffer-name prefix: a nested pipeline's buffers are its own
    explicit Ctx(DeviceCtx& dc) : d(dc) {}
    template <class T>
    T* up(const std::string& name, const std::vector<T>& v) {
        DevBuf& b = d.buf(pre + name);
        const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
        b.ensure(bytes);
        if (!v.empty()) {
            keep.emplace_back(reinterpret_cast<const uint8_t*>(v.data()),
                              reinterpret_cast<const uint8_t*>(v.data()) + v.size() * sizeof(T));
            SDSP_HIP_CHECK(hipMemcpyAsync(b.p, keep.back().data(), v.size() * sizeof(T), hipMemcpyHostToDevice, d.stream));
        }
        return b.as<T>();
    }
    // a host copy that lives until the context's queued work is done (async H2D source)
    template <class T>
    const void* keep_bytes(const std::vector<T>& v) {
        keep.emplace_back(reinterpret_cast<const uint8_t*>(v.data()),
                          reinterpret_cast<const uint8_t*>(v.data()) + v.size() * sizeof(T));
        return keep.back().data();
    }
    template <class T>
    T* dev(const std::string& name, size_t n) {
        DevBuf& b = d.buf(pre + name);
        b.ensure(std::max<size_t>(n * sizeof(T), 16));
        return b.as<T>();
    }
    template <class T>
    std::vector<T> down(const T* p, size_t n) {
        std::vector<T> v(n);
        if (n) SDSP_HIP_CHECK(hipMemcpyAsync(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost, d.stream));
        SDSP_HIP_CHECK(hipStreamSynchronize(d.stream));
        keep.clear();
        return v;
    }
    void sync() {
        SDSP_HIP_CHECK(hipStreamSynchronize(d.stream));
        keep.clear();
    }
};

struct Timers {
    hipEvent_t ev[16];
    int n = 0;
    DeviceCtx* d = nullptr;
    void init(DeviceCtx& dc) {
        d = &dc;
        for (auto& e : ev) SDSP_HIP_CHECK(hipEventCreate(&e));
    }
    void mark(int i, hipStream_t s = nullptr) { SDSP_HIP_CHECK(hipEventRecord(ev[i], s ? s : d->stream)); }
    double ms(int a, int b) {
        float t = 0.0f;
        if (hipEventElapsedTime(&t, ev[a], ev[b]) != hipSuccess) return 0.0;
        return t;
    }
    ~Timers() {
        if (d)
            for (auto& e : ev) (void)hipEventDestroy(e);
    }
};

struct TrackRes {
    int status = SDSP_OK;
    std::string err;
    float bpm = 0, bpm_conf = 0;
    int key_mode = 0, key_tonic = 0;
    float key_conf = 0, key_clarity = 0, stability = 0, duration = 0;
    float onset_consensus = 0;
    std::vector<float> beats, downs;
    int8_t mr_trig = -1, mr_used = -1, perc_trig = -1, perc_used = -1;
    bool has_cands = false;
    std::vector<sdsp_tempo_candidate> cands;
    int key_near = 0;  // block-folded key energies near a decision (KV_NEAR_* bits): rerun with the sequential fold
    bool key_rerun = false;  // that rerun has replaced the key fields
};

// Configuration support (everything the default path and its numeric knobs need).
std::string unsupported(const sdsp_config& c, uint32_t sr) {
    if (c.enable_normalization && c.normalization != SDSP_NORM_PEAK && c.normalization != SDSP_NORM_RMS &&
        c.normalization != SDSP_NORM_LOUDNESS)
        return "unknown normalization method";
    if (c.frame_size > (uint64_t)STFT_GEN_MAX || !stft_size_ok((int)c.frame_size))
        return "frame_size not a power of two in [64, 16384]";
    if (c.hop_size == 0 || c.hop_size > 8192) return "hop_size outside 1..8192";
    if ((c.enable_hpss_onsets || c.enable_tempogram_percussive_fallback) && c.hpss_margin > 16) return "hpss_margin > 16";
    if (!(c.min_bpm > 0.0f && c.max_bpm > c.min_bpm && c.bpm_resolution > 0.0f)) return "BPM range/resolution";
    if (c.force_legacy_bpm || c.enable_bpm_fusion) {  // k_legacy's fixed LDS lists
        int nc = 0;
        for (float b = c.min_bpm; b <= c.max_bpm + EPS && nc <= LG_COMB_MAX; b += c.bpm_resolution) nc++;
        if (nc > LG_COMB_MAX) return "legacy BPM: more than 2048 comb-filter candidates";
        const uint64_t hop = c.hop_size ? c.hop_size : 1;
        const float lmin = std::ceil((60.0f * (float)sr) / (c.max_bpm * (float)hop));
        const float lmax = std::floor((60.0f * (float)sr) / (c.min_bpm * (float)hop));
        if (lmax - lmin > (float)(2 * LG_AC_MAX - 4)) return "legacy BPM: autocorrelation lag range above 1020";
        if ((60.0f * (float)sr) / c.max_bpm < 1.0f) return "legacy BPM: period below one sample";
    }
    if (c.tempogram_superflux_max_filter_bins > (uint64_t)FT_KMAX) return "superflux_max_filter_bins > 8";
    if (c.enable_tempogram_mel_novelty && std::max<uint64_t>(c.tempogram_mel_n_mels, 4) > (uint64_t)FT_MELMAX)
        return "tempogram_mel_n_mels > 48";
    if (c.tempogram_mel_max_filter_bins > 16) return "tempogram_mel_max_filter_bins > 16";
    if (key_fft(c) > (uint64_t)STFT_GEN_MAX || !stft_size_ok((int)key_fft(c)))
        return "key STFT frame size not a power of two in [256, 16384]";
    if (c.enable_key_stft_override && c.key_stft_hop_size == 0) return "key_stft_hop_size 0";
    if (c.enable_key_hpss_harmonic && (c.key_hpss_time_margin > 16 || c.key_hpss_freq_margin > 16))
        return "key_hpss_time_margin / key_hpss_freq_margin > 16";
    if (c.key_spectrogram_smooth_margin > 31) return "key_spectrogram_smooth_margin > 31";
    if (c.enable_key_hpcp_whitening && c.key_hpcp_whitening_smooth_bins > 63) return "key_hpcp_whitening_smooth_bins > 63";
    if (c.key_hpcp_peaks_per_frame > (uint64_t)HP_KMAX) return "key_hpcp_peaks_per_frame > 32";
    if (c.key_hpcp_num_harmonics > (uint64_t)SUPPORT_HMAX) return "key_hpcp_num_harmonics > 8";
    if (c.enable_key_multi_scale && c.key_multi_scale_lengths_len > 8) return "more than 8 multi-scale key lengths";
    if (c.enable_ml_refinement) return "ML refinement";
    return "";
}

// One "tempo pass": STFT (2048, hop) -> features -> novelty -> tempograms -> candidate scoring,
// for a dense list of tracks.  Used for hop 512 (all tracks) and the escalation hops.
struct TempoPassIn {
    int hop;
    const float* samples;
    std::vector<uint64_t> src_off;  // per pass-track
    std::vector<float> gain_h;
    std::vector<uint64_t> n_trim;
    bool want_onsets;  // hop-512 pass: also spectral/HFC onset features (SFO)
    int top_n, gate, cand_cap;
    // a precomputed frame_size-point spectrogram (rows at the pass's frame prefix, stride s2_) and
    // its frame maxima: the STFT is skipped (the percussive tempogram fallback runs on the HPSS output)
    const float* mags_in = nullptr;
    const float* fmax_in = nullptr;
    // escalation hops over the hop-512 spectrogram (rows base_row0[t] + frame): 1 = hop 1024, every
    // frame is a hop-512 row (2v); 2 = hop 256, even frames are hop-512 rows, odd ones are computed
    int reuse = 0;
    const float* base_mags = nullptr;
    const float* base_fmax = nullptr;
    std::vector<uint64_t> base_row0;
    // also the hop-512 novelty multi_resolution.rs:680-694 gates its folds with (the combined
    // novelty with the configured weights, whatever the band-fusion setting; out.nov_mr)
    bool mr_nov = false;
};
struct TempoPassOut {
    std::vector<uint64_t> fpfx;  // frame prefix over the pass's tracks
    uint64_t total = 0;
    // device pointers (valid until the next pass with the same tag)
    float *mags = nullptr, *fmax = nullptr, *E = nullptr, *H = nullptr, *SFX = nullptr, *SFO = nullptr, *MEL = nullptr,
          *nov = nullptr, *nov_sum = nullptr, *cand = nullptr, *nov_mr = nullptr;
    uint64_t* d_fpfx = nullptr;
    TempoEst* est = nullptr;
    int* active = nullptr;
    std::vector<int> active_h;
    double stft_ms = 0, feat_ms = 0, tempo_ms = 0;
    uint64_t stft_launch = 0;
    uint64_t stft_frames = 0;
    double stft_bytes = 0;
};

}  // namespace

// ---------------------------------------------------------------------------------------
// debug_track_id dumps (src/lib.rs:461-487, 547-573, 1471-1538; multi_resolution.rs:304-403,
// 707-745, 845-857): the reference's eprintln! diagnostics, printed per analysed track in batch
// order from what the kernels computed (candidate lists, estimates, MrDbg / KeyDbg records).
struct Cand4 {
    float bpm, score, fft, acf;
};
struct TrackDbg {
    bool base = false;  // base tempogram estimate available (multi-resolution path)
    TempoEst est{};
    std::vector<Cand4> base_c;
    bool mr = false;  // escalated and every hop's tempogram succeeded
    std::vector<Cand4> c256, c512, c1024;
    TempoEst mr_est{};
    MrDbg md{};
    bool key = false;
    KeyOut ko{};
    KeyDbg kd{};
    float tuning = 0.0f;
};
const char* tf_str(bool b) { return b ? "true" : "false"; }
// cand_support (src/lib.rs:420-431) and lookup_nearest (multi_resolution.rs:281-292)
float cand_support(const std::vector<Cand4>& c, float bpm, float tol) {
    float b = 0.0f;
    for (const Cand4& x : c)
        if (sd_absf(x.bpm - bpm) <= tol) b = sd_maxf(b, x.score);
    return b;
}
float lookup_nearest_h(const std::vector<Cand4>& c, float bpm, float tol) {
    float bd = SD_INF_F, bs = 0.0f;
    for (const Cand4& x : c) {
        const float d = sd_absf(x.bpm - bpm);
        if (d <= tol && d < bd) {
            bd = d;
            bs = x.score;
        }
    }
    return bs;
}
std::string key_str(int key) {  // Key::name
    char b[8];
    sdsp_key_name(key < 12 ? 0 : 1, (uint32_t)(key % 12), b, sizeof b);
    return b;
}
void print_debug(const sdsp_config& c, const TrackDbg& d) {
    const unsigned id = c.debug_track_id;
    auto gt = [&]() {
        if (c.has_debug_gt_bpm) std::fprintf(stderr, "GT bpm: %.3f\n", (double)c.debug_gt_bpm);
    };
    const float tol = sd_maxf(2.0f, c.bpm_resolution);
    if (d.base) {
        const TempoEst& b = d.est;
        const float s_base = cand_support(d.base_c, b.bpm, tol), s_2x = cand_support(d.base_c, b.bpm * 2.0f, tol),
                    s_half = cand_support(d.base_c, b.bpm * 0.5f, tol);
        const bool fam = (s_2x > 0.0f && s_2x >= s_base * 0.90f) || (s_half > 0.0f && s_half >= s_base * 0.90f);
        const bool fold = b.bpm * 2.0f >= 170.0f && b.bpm * 2.0f <= 200.0f;
        const bool weak = b.agree == 0 || b.conf < 0.06f;
        std::fprintf(stderr, "\n=== DEBUG base tempogram (track_id=%u) ===\n", id);
        gt();
        std::fprintf(stderr, "base_est: bpm=%.2f conf=%.4f agree=%d (trap_low=%s trap_high=%s ambiguous=%s)\n",
                     (double)b.bpm, (double)b.conf, b.agree, tf_str(b.trap_low), tf_str(b.trap_high), tf_str(b.ambiguous));
        std::fprintf(stderr,
                     "ambiguity signals: family_competes=%s (s_base=%.4f s_2x=%.4f s_half=%.4f) weak_base=%s "
                     "fold_into_trap=%s\n",
                     tf_str(fam), (double)s_base, (double)s_2x, (double)s_half, tf_str(weak), tf_str(fold));
        if (!b.ambiguous) std::fprintf(stderr, "NOTE: multi-res not run (outside trap zones).\n");
    }
    if (d.mr) {
        const size_t top_n = std::max<uint64_t>(c.debug_top_n, 1);
        std::fprintf(stderr, "\n=== DEBUG multi-res (track_id=%u) ===\n", id);
        gt();
        auto top = [&](const char* label, const std::vector<Cand4>& v) {
            std::fprintf(stderr, "%s top-%zu:\n", label, top_n);
            for (size_t k = 0; k < v.size() && k < top_n; k++)
                std::fprintf(stderr, "  bpm=%7.2f score=%.4f\n", (double)v[k].bpm, (double)v[k].score);
        };
        top("hop=256", d.c256);
        top("hop=512", d.c512);
        top("hop=1024", d.c1024);
        if (c.has_debug_gt_bpm) {
            const float g = c.debug_gt_bpm;
            const float t512 = lookup_nearest_h(d.c512, g, tol), t256 = lookup_nearest_h(d.c256, g, tol),
                        t1024 = lookup_nearest_h(d.c1024, g, tol);
            const float d512 = lookup_nearest_h(d.c512, g * 2.0f, tol), d256 = lookup_nearest_h(d.c256, g * 2.0f, tol),
                        d1024 = lookup_nearest_h(d.c1024, g * 2.0f, tol);
            const float h512 = lookup_nearest_h(d.c512, g * 0.5f, tol), h256 = lookup_nearest_h(d.c256, g * 0.5f, tol),
                        h1024 = lookup_nearest_h(d.c1024, g * 0.5f, tol);
            std::fprintf(stderr, "Support near GT / family (lookup tol=%.2f):\n", (double)tol);
            std::fprintf(stderr, "  T     @512=%.4f @256=%.4f @1024=%.4f\n", (double)t512, (double)t256, (double)t1024);
            std::fprintf(stderr, "  2T    @512=%.4f @256=%.4f @1024=%.4f\n", (double)d512, (double)d256, (double)d1024);
            std::fprintf(stderr, "  T/2   @512=%.4f @256=%.4f @1024=%.4f\n", (double)h512, (double)h256, (double)h1024);
            const float w512 = c.tempogram_multi_res_w512, w256 = c.tempogram_multi_res_w256,
                        w1024 = c.tempogram_multi_res_w1024, dt = c.tempogram_multi_res_double_time_512_factor;
            const float h_t = w512 * t512 + w256 * t256 + w1024 * (t1024 + c.tempogram_multi_res_structural_discount * d1024);
            float h_2t = w512 * (dt * t512 + (1.0f - dt) * d512) + w256 * d256 + w1024 * d1024;
            float h_h = w512 * (dt * t512 + (1.0f - dt) * h512) + w256 * h256 + w1024 * h1024;
            const float eps = 1e-6f;
            const float r2 = (d256 + eps) / (t256 + eps), rh = (h1024 + eps) / (t1024 + eps);
            if (r2 < 1.10f) h_2t *= 0.75f;
            if (r2 < 1.00f) h_2t *= 0.75f;
            if (rh < 1.10f) h_h *= 0.75f;
            if (rh < 1.00f) h_h *= 0.75f;
            struct L {
                float bpm, s;
                const char* tag;
            };
            std::vector<L> loc = {{g, h_t, "T"}, {g * 2.0f, h_2t, "2T"}, {g * 0.5f, h_h, "T/2"}};
            std::vector<L> keep;
            for (const L& l : loc)
                if (l.bpm >= c.min_bpm && l.bpm <= c.max_bpm) keep.push_back(l);
            for (L& l : keep) {
                if (l.bpm > 210.0f) l.s *= 0.80f;
                else if (l.bpm > 180.0f) l.s *= 0.90f;
                else if (l.bpm < 60.0f) l.s *= 0.92f;
            }
            std::stable_sort(keep.begin(), keep.end(), [](const L& a, const L& b) { return a.s > b.s; });
            std::fprintf(stderr, "Fusion scores (T anchored at GT, after guardrails+prior):\n");
            for (const L& l : keep) std::fprintf(stderr, "  %3s bpm=%7.2f score=%.4f\n", l.tag, (double)l.bpm, (double)l.s);
            if (keep.size() >= 2)
                std::fprintf(stderr, "  margin(best-second)=%.4f (threshold=%.4f)\n", (double)(keep[0].s - keep[1].s),
                             (double)c.tempogram_multi_res_margin_threshold);
            std::fprintf(stderr, "  ratio_2T_256=%.3f ratio_half_1024=%.3f (guardrails)\n", (double)r2, (double)rh);
        }
        const MrDbg& m = d.md;
        if (m.fd)
            std::fprintf(stderr, "DEBUG fold-down (track_id=%u): %.2f -> %.2f (support ratio %.3f, agree %d->%d).\n", id,
                         (double)m.fd_from, (double)m.fd_to, (double)m.fd_ratio, m.fd_a0, m.fd_a1);
        if (m.fu)
            std::fprintf(stderr, "DEBUG fold-up (track_id=%u): %.2f -> %.2f (support ratio %.3f, agree %d->%d).\n", id,
                         (double)m.fu_from, (double)m.fu_to, (double)m.fu_ratio, m.fu_a0, m.fu_a1);
        if (m.tf) {
            static const char* lab[5] = {"T", "3/2", "2/3", "4/3", "3/4"};
            std::fprintf(stderr,
                         "DEBUG triplet-family (track_id=%u): %.2f -> %.2f (%s, support %.3f->%.3f, align %.3f->%.3f)\n",
                         id, (double)m.tf_from, (double)m.tf_to, lab[m.tf_label < 0 || m.tf_label > 4 ? 0 : m.tf_label],
                         (double)m.tf_sup0, (double)m.tf_sup1, (double)m.tf_al0, (double)m.tf_al1);
        }
        std::fprintf(stderr, "\n=== DEBUG multi-res decision (track_id=%u) ===\n", id);
        gt();
        std::fprintf(stderr, "base_est: bpm=%.2f conf=%.4f agree=%d\n", (double)d.est.bpm, (double)d.est.conf, d.est.agree);
        std::fprintf(stderr, "mr_est:   bpm=%.2f conf=%.4f agree=%d\n", (double)d.mr_est.bpm, (double)d.mr_est.conf,
                     d.mr_est.agree);
        std::fprintf(stderr, "ambiguous(trap_low||trap_high)=%s\n", tf_str(d.est.ambiguous));
        std::fprintf(stderr, "rel=%.3f family_related=%s forbid_promote_high=%s\n", (double)m.rel, tf_str(m.fam),
                     tf_str(m.forbid));
        std::fprintf(stderr, "mr_better=%s used_mr=%s\n", tf_str(m.better), tf_str(m.better));
    }
    if (d.key) {
        const KeyDbg& k = d.kd;
        std::fprintf(stderr, "\n=== DEBUG key (track_id=%u) ===\n", id);
        std::fprintf(stderr,
                     "key=%s conf=%.4f clarity=%.4f frames=%d used_frames=%d soft_mapping=%s sigma=%.3f harmonic_mask=%s "
                     "mask_p=%.2f tuning=%.4f time_smooth=%s margin=%llu edge_trim=%s trim_frac=%.2f\n",
                     key_str(d.ko.mode * 12 + d.ko.tonic).c_str(), (double)d.ko.conf, (double)d.ko.clarity, k.frames, k.used,
                     tf_str(c.soft_chroma_mapping), (double)c.soft_mapping_sigma, tf_str(c.enable_key_harmonic_mask),
                     (double)c.key_harmonic_mask_power, (double)d.tuning, tf_str(c.enable_key_spectrogram_time_smoothing),
                     (unsigned long long)c.key_spectrogram_smooth_margin, tf_str(c.enable_key_edge_trim),
                     (double)c.key_edge_trim_fraction);
        // top_keys: the first three of the final table; the chosen key replaces the third when it is
        // not among them (detector.rs:506-510)
        std::vector<std::pair<int, float>> tk;
        for (int q = 0; q < 3; q++) tk.push_back({k.order[q], k.tab[q]});
        bool in = false;
        for (const auto& e : tk) in |= e.first == k.key;
        if (!in)
            for (int q = 3; q < 24; q++)
                if (k.order[q] == k.key) tk.back() = {k.key, k.tab[q]};
        std::string line;
        for (size_t q = 0; q < tk.size(); q++) {
            char b[64];
            std::snprintf(b, sizeof b, "%s%s:%.4f", q ? ", " : "", key_str(tk[q].first).c_str(), (double)tk[q].second);
            line += b;
        }
        std::fprintf(stderr, "top_keys: %s\n", line.c_str());
        static const char* notes[12] = {"C", "C#", "D", "D#", "E", "F", "F#", "G", "G#", "A", "A#", "B"};
        std::vector<int> pcs(12);
        for (int q = 0; q < 12; q++) pcs[q] = q;
        std::stable_sort(pcs.begin(), pcs.end(), [&](int a, int b) { return k.agg[a] > k.agg[b]; });
        line.clear();
        for (int q = 0; q < 6; q++) {
            char b[64];
            std::snprintf(b, sizeof b, "%s%s:%.3f", q ? ", " : "", notes[pcs[q]], (double)k.agg[pcs[q]]);
            line += b;
        }
        std::fprintf(stderr, "top_pitch_classes(weighted): %s\n", line.c_str());
    }
}

// ---------------------------------------------------------------------------------------
class Pipeline {
   public:
    Pipeline(DeviceCtx& d, const sdsp_config& cfg, uint32_t sr, int stages = SDSP_STAGES_FULL, bool exact_energy = false,
             bool key_only = false, bool nested = false)
        : c_(d),
          d_(d),
          cfg_(cfg),
          sr_(sr),
          bpm_only_(stages == SDSP_STAGES_BPM_ONLY),
          exact_energy_(exact_energy),
          key_only_(key_only),
          nested_(nested),
          fs_((int)std::min<uint64_t>(cfg.frame_size, STFT_GEN_MAX)),
          nb_(fs_ / 2 + 1),
          s2_(base_stride(fs_)),
          kfs_((int)std::min<uint64_t>(key_fft(cfg), STFT_GEN_MAX)),
          khop_((int)std::min<uint64_t>(std::max<uint64_t>(key_hop(cfg), 1), INT32_MAX)),
          ks_(base_stride(kfs_)) {
        if (nested_) c_.pre = "X.";
    }

    void run(const float* d_samples, const std::vector<uint64_t>& in_off, const std::vector<uint64_t>& n_raw,
             std::vector<TrackRes>& res);

   private:
    Ctx c_;
    DeviceCtx& d_;
    const sdsp_config& cfg_;
    uint32_t sr_;
    // SDSP_STAGES_BPM_ONLY: the tempo path alone (src/lib.rs:86-910); the key
    // stream and the beat grid are not run, their result fields keep their defaults
    bool bpm_only_ = false;
    // the key path with the reference's sequential frame-energy fold (k_mask_r / k_hpcp) even where
    // the band-limited mask applies: run_locked's rerun of tracks whose key vote was near a decision
    bool exact_energy_ = false;
    // the key path alone (with exact_energy_: the rerun): front end, key stream, key fields only
    bool key_only_ = false;
    // a rerun started from inside the main pass (rerun_near): its buffers carry the prefix "X."
    // and its key path runs on the main stream, in that stream's slack beside the key stream
    bool nested_ = false;
    // the sub-batch being run is the call's last (its key vote runs alone at the tail)
    bool last_sub_ = false;
    uint64_t reruns_ = 0;
    double rerun_ms_ = 0.0;
    void rerun_near(const float* d_samples, const std::vector<uint64_t>& in_off, const std::vector<uint64_t>& n_raw,
                    const std::vector<size_t>& near, std::vector<TrackRes>& res);
    // the tempo path's STFT: frame size (AnalysisConfig::frame_size), bins, row stride
    const int fs_, nb_, s2_;
    // the key path's STFT: frame size, hop, row stride (key_fft / key_hop)
    const int kfs_, khop_, ks_;
    sdsp_stage_times times_{};
    // RMS / LUFS: gains (and LUFS status) of every track, folded once for the whole batch
    // before the sub-batches (the fold is a per-track sequential latency, not a throughput)
    std::vector<float> loud_gain_;
    std::vector<int> loud_stat_;

    void loudness_prepass(const float* d_samples, const std::vector<uint64_t>& in_off,
                          const std::vector<uint64_t>& n_raw, std::vector<TrackRes>& res);

    void sub_batch(const float* d_samples, const std::vector<uint64_t>& in_off, const std::vector<uint64_t>& n_raw,
                   const std::vector<int>& idx, std::vector<TrackRes>& res);
    // Late key join: a sub-batch's key results are read after the next sub-batch's tempo path is
    // queued, so the key stream's tail (mask, HPCP, vote) runs beside that tempo path instead of
    // holding the main stream back.  Uploads read by the key stream and the key output live in
    // per-parity buffers (E0.*, E1.*); the key stream itself is in order, so its big buffers are
    // shared.
    // The band path's state of a sub-batch for the exact rerun in place (rerun_tail): its key
    // spectrogram (band masked in place, every other bin the STFT's), its chroma and vote buffers.
    // Valid for the call's last sub-batch only (the next sub-batch's key stream reuses them).
    struct KeyTail {
        bool ok = false;
        float* mags8 = nullptr;
        uint64_t* d_kpfx = nullptr;
        std::vector<uint64_t> kpfx, kseg;  // frame and segment-scratch prefixes over the key tracks
        float* d_part = nullptr;
        uint64_t total8 = 0;
        int st_lo = 0, st_hi = -1, B8 = 0;
        HpcpParams hp{};
        const HarmEntry* d_ht = nullptr;
        float *d_chroma = nullptr, *d_energy = nullptr, *d_cs = nullptr, *d_w = nullptr, *d_sscr = nullptr;
        const float* d_tpl = nullptr;
        KeyParams kp{};
    };
    struct KeyPending {
        std::unique_ptr<Timers> kt;
        KeyOut* d_kout = nullptr;
        std::vector<size_t> at;  // result slot of each key track
        KeyTail tail;
    };
    std::unique_ptr<KeyPending> key_pending_;
    std::unique_ptr<KeyPending> tail_;  // the last sub-batch's pending join, kept for rerun_tail
    int sb_parity_ = 0;
    std::vector<size_t> finish_key(std::vector<TrackRes>& res, bool keep_tail = false);
    void rerun_tail(const std::vector<size_t>& near, std::vector<TrackRes>& res);
    void tempo_pass(const std::string& tag, const TempoPassIn& in, TempoPassOut& out);
    void legacy_select(const TempoPassIn& bin, const uint32_t* d_onsets, const uint64_t* d_on_off, const int* d_on_n,
                       const std::vector<int>& R, const std::vector<int>& idx, std::vector<TrackRes>& res,
                       std::vector<float>& fbpm_h, std::vector<float>& fconf_h, float* d_fbpm, float* d_fconf);
};

void Pipeline::run(const float* d_samples, const std::vector<uint64_t>& in_off, const std::vector<uint64_t>& n_raw,
                   std::vector<TrackRes>& res) {
    const size_t T = n_raw.size();
    res.assign(T, TrackRes{});
    std::string why = unsupported(cfg_, sr_);
    if (why.empty()) why = unsupported_sr(cfg_, sr_);
    for (size_t i = 0; i < T; i++) {
        if (n_raw[i] == 0) {
            res[i].status = SDSP_ERR_INVALID_INPUT;
            res[i].err = "Invalid input: Empty audio samples";
        } else if (sr_ == 0) {
            res[i].status = SDSP_ERR_INVALID_INPUT;
            res[i].err = "Invalid input: Invalid sample rate";
        } else if (!why.empty()) {
            res[i].status = SDSP_ERR_NOT_IMPLEMENTED;
            res[i].err = "Not implemented: " + why;
        }
    }
    // Sub-batches under an HBM budget (bytes per track estimated from its raw length): what is
    // free now plus what this context already holds (its buffers are reused), less headroom
    // for the grow-only buffers' 1/8 slack.  SDSP_HBM_BUDGET_GB overrides.
    double budget = 64e9;
    {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
            double held = 0;  // (a nested rerun's "X." buffers are not this pipeline's to reuse)
            for (auto& kv : d_.bufs)
                if (kv.first.compare(0, c_.pre.size(), c_.pre) == 0 && (!c_.pre.empty() || kv.first.compare(0, 2, "X.") != 0))
                    held += (double)kv.second->bytes;
            budget = std::max(4e9, ((double)fr + held) * 0.80 / 1.125);
        }
        // schedule knob (sdsp_debug_set_schedule): the tests' several-sub-batch paths
        if (const double gb = test_hooks().hbm_budget_gb.load(); gb > 0.0) budget = std::max(1.0, gb) * 1e9;
    }
    const uint64_t hop = cfg_.hop_size, khop = (uint64_t)khop_;
    std::vector<int> cur;
    double acc = 0;
    auto flush = [&]() {
        if (!cur.empty()) sub_batch(d_samples, in_off, n_raw, cur, res);
        cur.clear();
        acc = 0;
    };
    times_ = sdsp_stage_times{};
    last_sub_ = false;
    auto t0 = std::chrono::steady_clock::now();
    if (cfg_.enable_normalization && cfg_.normalization != SDSP_NORM_PEAK && why.empty())
        loudness_prepass(d_samples, in_off, n_raw, res);
    // equal shares: the fewest sub-batches that fit the budget, each near total / count (a
    // short last sub-batch runs at a fraction of the chip)
    std::vector<double> need(T, 0.0);
    double total_need = 0;
    for (size_t i = 0; i < T; i++) {
        if (res[i].status != SDSP_OK) continue;
        const double n = (double)n_raw[i];
        need[i] = n / hop * (s2_ * 4.0 * 1.3 + 4 * 70.0) + (bpm_only_ ? 0.0 : n / khop * ks_ * 4.0) +
                  (n / 256 + n / 1024) * s2_ * 4.0 + 1e6;
        if (cfg_.enable_hpss_onsets || cfg_.enable_tempogram_percussive_fallback)  // H, P ping-pong + a copy
            need[i] += n / hop * s2_ * 4.0 * 5.0;
        if (cfg_.enable_key_hpss_harmonic && !bpm_only_) need[i] += n / khop * 1024.0 * 4.0;
        if (cfg_.enable_tempogram_multi_resolution && hop != 512) need[i] += n / 512 * s2_ * 4.0 * 1.3;
        total_need += need[i];
    }
    const double parts = std::max(1.0, std::ceil(total_need / budget));
    const double share = total_need / parts;
    double cum = 0;
    int part = 0;
    for (size_t i = 0; i < T; i++) {
        if (res[i].status != SDSP_OK) continue;
        // a track belongs to the share its midpoint falls in
        const int p = (int)std::min(parts - 1.0, std::floor((cum + 0.5 * need[i]) / share));
        if (!cur.empty() && (p != part || acc + need[i] > budget)) flush();
        part = p;
        cur.push_back((int)i);
        acc += need[i];
        cum += need[i];
    }
    last_sub_ = true;
    flush();
    last_sub_ = false;
    // the last sub-batch's near tracks: rerun in place when its band-path buffers are intact,
    // otherwise by run_locked
    rerun_tail(finish_key(res, true), res);
    times_.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    times_.key_reruns = reruns_;  // in-flight reruns (rerun_near), their time inside total_ms
    times_.rerun_ms = rerun_ms_;
    d_.last = times_;
}

void Pipeline::loudness_prepass(const float* d_samples, const std::vector<uint64_t>& in_off,
                                const std::vector<uint64_t>& n_raw, std::vector<TrackRes>& res) {
    const size_t T = n_raw.size();
    loud_gain_.assign(T, 1.0f);
    loud_stat_.assign(T, 0);
    const LoudnessParams lp = loudness_params(cfg_.normalization, sr_);
    std::vector<uint64_t> off, nr, cpfx(1, 0);
    std::vector<size_t> at;
    for (size_t i = 0; i < T; i++) {
        if (res[i].status != SDSP_OK) continue;
        if (lp.method == 2 && lp.block == 0) {  // calculate_lufs :199-204
            res[i].status = SDSP_ERR_INVALID_INPUT;
            res[i].err = "Invalid input: Sample rate too low for LUFS calculation";
            continue;
        }
        at.push_back(i);
        off.push_back(in_off[i]);
        nr.push_back(n_raw[i]);
        cpfx.push_back(cpfx.back() + (n_raw[i] + PK_CH - 1) / PK_CH);
    }
    const int L = (int)at.size();
    if (L == 0) return;
    uint64_t* d_off = c_.up("L.off", off);
    uint64_t* d_nr = c_.up("L.nr", nr);
    uint64_t* d_cpfx = c_.up("L.cpfx", cpfx);
    unsigned int* d_peak = c_.dev<unsigned int>("L.peak", (size_t)L);
    float* d_gain = c_.dev<float>("L.gain", (size_t)L);
    int* d_stat = c_.dev<int>("L.stat", (size_t)L);
    launch_loudness_gain(d_samples, d_off, d_nr, d_cpfx, L, cpfx.back(),
                         c_.dev<unsigned int>("L.peakchunk", std::max<uint64_t>(cpfx.back(), 1)), d_peak, lp, d_gain,
                         d_stat, d_.stream);
    SDSP_HIP_CHECK(hipGetLastError());
    const std::vector<float> g = c_.down(d_gain, (size_t)L);
    const std::vector<int> st = c_.down(d_stat, (size_t)L);
    for (int k = 0; k < L; k++) {
        loud_gain_[at[(size_t)k]] = g[(size_t)k];
        loud_stat_[at[(size_t)k]] = st[(size_t)k];
    }
}

// The legacy estimate of every track from its beat-tracking onsets (on_legacy == on_beat,
// src/lib.rs:176-291), then force_legacy_bpm / enable_bpm_fusion's choice (src/lib.rs:814-892).
// ACF scratch: M = next_pow2(2L) complex per buffer, L <= (n_trim - 1) / hop + 1.
void Pipeline::legacy_select(const TempoPassIn& bin, const uint32_t* d_onsets, const uint64_t* d_on_off,
                             const int* d_on_n, const std::vector<int>& R, const std::vector<int>& idx,
                             std::vector<TrackRes>& res, std::vector<float>& fbpm_h, std::vector<float>& fconf_h,
                             float* d_fbpm, float* d_fconf) {
    hipStream_t st = d_.stream;
    const int NR = (int)R.size();
    const uint64_t hop = (uint64_t)bin.hop;
    std::vector<uint64_t> soff((size_t)NR), scap((size_t)NR);
    uint64_t tot = 0, mmax = 4;
    for (int i = 0; i < NR; i++) {
        const uint64_t n = bin.n_trim[(size_t)i];
        const uint64_t L = (n ? n - 1 : 0) / hop + 1;
        uint64_t M = 1;
        while (M < 2 * L) M <<= 1;
        scap[(size_t)i] = M;
        soff[(size_t)i] = tot;
        tot += 2 * M;
        mmax = std::max(mmax, M);
    }
    LegacyParams P{};
    P.sr = (int)sr_;
    P.hop = (int)hop;
    P.min_bpm = cfg_.min_bpm;
    P.max_bpm = cfg_.max_bpm;
    P.res = cfg_.bpm_resolution;
    P.guard = cfg_.enable_legacy_bpm_guardrails ? 1 : 0;
    {  // LegacyBpmGuardrails::clamp_sane (period/mod.rs:88-121)
        const float pmn = cfg_.legacy_bpm_preferred_min, pmx = cfg_.legacy_bpm_preferred_max;
        const float smn = cfg_.legacy_bpm_soft_min, smx = cfg_.legacy_bpm_soft_max;
        P.g[0] = sd_minf(pmn, pmx);
        P.g[1] = sd_maxf(pmn, pmx);
        P.g[2] = sd_minf(sd_minf(smn, smx), P.g[0]);
        P.g[3] = sd_maxf(sd_maxf(smn, smx), P.g[1]);
        const float mul[3] = {cfg_.legacy_bpm_conf_mul_preferred, cfg_.legacy_bpm_conf_mul_soft,
                              cfg_.legacy_bpm_conf_mul_extreme};
        for (int k = 0; k < 3; k++) P.g[4 + k] = sd_isfinite_f(mul[k]) ? sd_maxf(mul[k], 0.0f) : 0.0f;
    }
    FftTables& tb = d_.tables((int)(2 * mmax), false);
    cx* scr = c_.dev<cx>("G.acf", tot);
    LegacyOut* d_lo = c_.dev<LegacyOut>("G.out", (size_t)NR);
    launch_legacy(d_onsets, d_on_off, d_on_n, NR, c_.up("G.soff", soff), c_.up("G.scap", scap), scr, tb.tw.as<cx>(),
                  (int)mmax, P, d_lo, st);
    SDSP_HIP_CHECK(hipGetLastError());
    const std::vector<LegacyOut> lo = c_.down(d_lo, (size_t)NR);
    for (int i = 0; i < NR; i++) {
        TrackRes& r = res[(size_t)idx[(size_t)R[(size_t)i]]];
        const LegacyOut& l = lo[(size_t)i];
        if (l.ok < 0) {  // estimate_bpm_with_guardrails(...)? propagates (src/lib.rs:315, 324)
            r.status = SDSP_ERR_PROCESSING;
            r.err = l.ok == -1 ? "Processing error: Signal too short for autocorrelation"
                               : "Processing error: legacy BPM scratch too small";
            continue;
        }
        const bool has = l.ok > 0;
        float& bpm = fbpm_h[(size_t)i];
        float& conf = fconf_h[(size_t)i];
        if (cfg_.force_legacy_bpm) {
            bpm = has ? l.bpm : 0.0f;
            conf = has ? l.conf : 0.0f;
            continue;
        }
        // fusion: the tempogram BPM is kept; legacy only moves its confidence
        const float t_bpm = bpm, t_conf = conf;
        const float l_bpm = has ? l.bpm : 0.0f;
        const float l_conf = sd_clampf(has ? l.conf : 0.0f, 0.0f, 1.0f);
        if (t_bpm <= 0.0f) {
            bpm = has ? l.bpm : 0.0f;
            conf = has ? l.conf : 0.0f;
            continue;
        }
        float c = sd_clampf(t_conf, 0.0f, 1.0f);
        bool agree = false;
        if (l_bpm > 0.0f) {
            const float d[5] = {sd_absf(l_bpm - t_bpm), sd_absf(l_bpm - (t_bpm * 0.5f)), sd_absf(l_bpm - (t_bpm * 2.0f)),
                                sd_absf(l_bpm - (t_bpm * (2.0f / 3.0f))), sd_absf(l_bpm - (t_bpm * (3.0f / 2.0f)))};
            for (float v : d) agree |= v <= 2.0f;
        }
        if (agree)
            c = sd_clampf(c + 0.12f * l_conf, 0.0f, 1.0f);
        else if (l_bpm > 0.0f)
            c = sd_clampf(c * 0.90f, 0.0f, 1.0f);
        conf = c;
    }
    SDSP_HIP_CHECK(hipMemcpyAsync(d_fbpm, c_.keep_bytes(fbpm_h), (size_t)NR * sizeof(float), hipMemcpyHostToDevice, st));
    SDSP_HIP_CHECK(hipMemcpyAsync(d_fconf, c_.keep_bytes(fconf_h), (size_t)NR * sizeof(float), hipMemcpyHostToDevice, st));
}

void Pipeline::tempo_pass(const std::string& tag, const TempoPassIn& in, TempoPassOut& o) {
    const int P_T = (int)in.src_off.size();
    const int FS = fs_, hop = in.hop;
    // frames per pass-track
    o.fpfx.assign((size_t)P_T + 1, 0);
    std::vector<uint64_t> tpfx((size_t)P_T + 1, 0);
    o.active_h.assign((size_t)P_T, 0);
    for (int t = 0; t < P_T; t++) {
        const uint64_t n = in.n_trim[(size_t)t];
        const uint64_t F = n >= (uint64_t)FS ? (n - FS) / (uint64_t)hop + 1 : 0;
        o.fpfx[(size_t)t + 1] = o.fpfx[(size_t)t] + F;
        tpfx[(size_t)t + 1] = tpfx[(size_t)t] + (F + FT_STEP - 1) / FT_STEP;
        o.active_h[(size_t)t] = F >= 2;
    }
    const uint64_t total = o.fpfx[(size_t)P_T];
    o.total = total;
    o.d_fpfx = c_.up(tag + "fpfx", o.fpfx);
    uint64_t* d_tpfx = c_.up(tag + "tpfx", tpfx);
    uint64_t* d_src = c_.up(tag + "src", in.src_off);
    float* d_gain = c_.up(tag + "gain", in.gain_h);
    o.active = c_.up(tag + "active", o.active_h);
    // STFT
    FftTables& tb = d_.tables(FS, true);
    Timers tm;
    tm.init(d_);
    tm.mark(0);
    RowMap rm{};
    uint64_t stft_frames = 0;
    if (in.mags_in) {
        o.mags = const_cast<float*>(in.mags_in);
        o.fmax = const_cast<float*>(in.fmax_in);
    } else if (in.reuse == 1) {  // hop 1024: nothing to compute
        o.mags = nullptr;
        o.fmax = nullptr;
        rm = RowMap{in.base_mags, in.base_mags, in.base_fmax, in.base_fmax, c_.up(tag + "brow", in.base_row0), nullptr,
                    2, 4, 4};
    } else if (in.reuse == 2) {  // hop 256: the odd frames, as a hop-512 STFT from sample 256
        std::vector<uint64_t> opfx((size_t)P_T + 1, 0), osrc((size_t)P_T);
        for (int t = 0; t < P_T; t++) {
            opfx[(size_t)t + 1] = opfx[(size_t)t] + (o.fpfx[(size_t)t + 1] - o.fpfx[(size_t)t]) / 2;
            osrc[(size_t)t] = in.src_off[(size_t)t] + (uint64_t)hop;
        }
        stft_frames = opfx[(size_t)P_T];
        o.mags = c_.dev<float>(tag + "mags", std::max<uint64_t>(stft_frames, 1) * s2_);
        o.fmax = c_.dev<float>(tag + "fmax", std::max<uint64_t>(stft_frames, 1));
        uint64_t* d_opfx = c_.up(tag + "opfx", opfx);
        const std::vector<uint64_t> ostr = stft_strips(opfx);
        launch_stft(FS, true, in.samples, d_opfx, P_T, stft_frames, c_.up(tag + "osrc", osrc), d_gain, 2 * hop,
                    tb.window.as<float>(), stft_twp(tb, FS, true), stft_rtp(tb, FS, true), o.mags, d_opfx, s2_, o.fmax,
                    d_.stream, c_.up(tag + "ostrip", ostr), ostr.back(), c_.dev<uint32_t>(tag + "redo", stft_frames + 1));
        SDSP_HIP_CHECK(hipGetLastError());
        rm = RowMap{in.base_mags, o.mags, in.base_fmax, o.fmax, c_.up(tag + "brow", in.base_row0), d_opfx, 0, 1, 1};
    } else {
        o.mags = c_.dev<float>(tag + "mags", total * s2_);
        o.fmax = c_.dev<float>(tag + "fmax", total);
        const std::vector<uint64_t> str = stft_strips(o.fpfx);
        launch_stft(FS, true, in.samples, o.d_fpfx, P_T, total, d_src, d_gain, hop, tb.window.as<float>(),
                    stft_twp(tb, FS, true), stft_rtp(tb, FS, true), o.mags, o.d_fpfx, s2_, o.fmax, d_.stream,
                    c_.up(tag + "strip", str), str.back(), c_.dev<uint32_t>(tag + "redo", total + 1));
        SDSP_HIP_CHECK(hipGetLastError());
        stft_frames = total;
    }
    if (in.mags_in || in.reuse == 0) rm = RowMap{o.mags, o.mags, o.fmax, o.fmax, o.d_fpfx, nullptr, 1, 2, 2};
    tm.mark(1);
    o.stft_launch = stft_frames ? 1 : 0;
    o.stft_frames = stft_frames;
    if (stft_frames) {
        double inb = 0;
        for (int t = 0; t < P_T; t++) inb += 4.0 * (double)in.n_trim[(size_t)t];
        o.stft_bytes = inb + 4.0 * (double)stft_frames * (double)nb_;
    }
    // features
    const int B = nb_;
    FeatParams fp{};
    fp.B = B;
    fp.stride = s2_;
    fp.K = (int)std::max<uint64_t>(cfg_.tempogram_superflux_max_filter_bins, 1);
    const float fres = (float)sr_ / (float)((B - 1) * 2);
    const int b0 = std::min(1, B - 1);
    const int bl = std::max(hz_to_bin(cfg_.tempogram_band_low_max_hz, fres, B), b0);
    const int bm = std::max(hz_to_bin(cfg_.tempogram_band_mid_max_hz, fres, B), bl + 1);
    int bh = cfg_.tempogram_band_high_max_hz > 0.0f ? std::max(hz_to_bin(cfg_.tempogram_band_high_max_hz, fres, B), bm + 1) : B;
    bh = std::min(bh, B);
    const float wb[4] = {cfg_.tempogram_band_w_full, cfg_.tempogram_band_w_low, cfg_.tempogram_band_w_mid,
                         cfg_.tempogram_band_w_high};
    const int bs_[4] = {0, b0, bl, bm}, be_[4] = {B, bl, bm, bh};
    const bool band_cfg = cfg_.enable_tempogram_band_fusion || cfg_.enable_tempogram_mel_novelty ||
                          cfg_.tempogram_band_consensus_bonus > 0.0f;  // use_aux_variants (src/lib.rs:375-377)
    for (int v = 0; v < 4; v++) {
        fp.bs[v] = std::min(bs_[v], B);
        fp.be[v] = std::min(be_[v], B);
        if (v == 0)
            fp.band_on[v] = 1;
        else
            fp.band_on[v] = band_cfg && cfg_.enable_tempogram_band_fusion && sd_isfinite_f(wb[v]) && wb[v] > 0.0f &&
                            be_[v] > bs_[v] + 1 && fp.be[v] > fp.bs[v] + 1;
    }
    const bool mel_on = band_cfg && cfg_.enable_tempogram_mel_novelty;
    std::string merr;
    MelTable mt = mel_table(sr_, B, (int)cfg_.tempogram_mel_n_mels, cfg_.tempogram_mel_fmin_hz, cfg_.tempogram_mel_fmax_hz,
                            &merr);
    if (!merr.empty()) throw HipError(merr);
    fp.n_mels = mel_on ? mt.n_mels : 0;
    std::vector<MelPlan> mplan = mel_plan(mt, B, &merr);
    if (!merr.empty()) throw HipError(merr);
    MelPlan* d_mplan = c_.up(tag + "melplan", mplan);
    // k_features' per-chunk flags (8-bin chunks of the <8, 16, 4> walk; see FeatParams)
    {
        auto band_of = [&](int b) {
            int v = 0;
            for (int q = 3; q >= 1; q--)
                if (fp.band_on[q] && b >= fp.bs[q] && b < fp.be[q]) v = q;
            return v;
        };
        std::vector<int> cf((size_t)(B + 7) / 8 + 1, 0);
        std::vector<MelChunk> mc((size_t)(B + 7) / 8 + 1, MelChunk{});
        for (int c0 = 0; c0 < B; c0 += 8) {
            const int v0 = band_of(c0);
            bool fast = fp.K == 4 && c0 + 8 <= B, mel = false, mel_ok = true, mel_reg = true;
            MelChunk& m = mc[(size_t)c0 / 8];
            for (int j = 0; j < 8; j++) m.bf[j] = (float)(c0 + j);
            for (int b = c0; fast && b < c0 + 8; b++) {
                const int v = band_of(b);
                if (v != v0) fast = false;
                if (v) {
                    const int lo = b - fp.K < 0 ? 0 : b - fp.K, hi = b + fp.K + 1 < B ? b + fp.K + 1 : B;
                    if (lo < fp.bs[v] || hi > fp.be[v]) fast = false;
                }
                if (fp.n_mels > 0) {
                    const MelPlan& q = mplan[(size_t)b];
                    if (q.nflush != 0 || q.w0 != 0.0f || q.w1 != 0.0f) mel = true;
                    if (q.nflush < 0 || q.nflush > 3 || (q.s0 & ~1) || (q.s1 & ~1)) mel_ok = false;
                    if ((q.w0 != 0.0f && q.s0 != 0) || (q.w1 != 0.0f && q.s1 != 1)) mel_reg = false;
                    const int j = b - c0;
                    m.bits |= (uint32_t)(q.nflush & 3) << (4 * j) | (uint32_t)(q.s0 & 1) << (4 * j + 2) |
                              (uint32_t)(q.s1 & 1) << (4 * j + 3);
                    m.w0[j] = q.w0;
                    m.w1[j] = q.w1;
                }
            }
            cf[(size_t)c0 / 8] = v0 | (fast && !mel ? FT_CHUNK_FAST : 0) | (fast && mel && mel_ok ? FT_CHUNK_MEL : 0) |
                                 (fast && mel && mel_ok && mel_reg ? FT_CHUNK_MELREG : 0);
        }
        fp.chunk_flags = c_.up(tag + "ftchunk", cf);
        fp.mel_chunks = c_.up(tag + "ftmelchunk", mc);
    }
    o.E = c_.dev<float>(tag + "E", 4 * total);
    o.H = c_.dev<float>(tag + "H", 4 * total);
    o.SFX = c_.dev<float>(tag + "SFX", 4 * total);
    o.SFO = c_.dev<float>(tag + "SFO", total);
    o.MEL = c_.dev<float>(tag + "MEL", std::max<uint64_t>(total * (uint64_t)std::max(fp.n_mels, 1), 1));
    launch_features(rm, o.d_fpfx, d_tpfx, P_T, tpfx[(size_t)P_T], fp, d_mplan, o.E, o.H, o.SFX, o.SFO,
                    o.MEL, total, d_.stream);
    SDSP_HIP_CHECK(hipGetLastError());
    // novelty
    NovParams np{};
    if (band_cfg) {
        np.ws = sd_maxf(cfg_.tempogram_novelty_w_spectral, 0.0f);
        np.we = sd_maxf(cfg_.tempogram_novelty_w_energy, 0.0f);
        np.wh = sd_maxf(cfg_.tempogram_novelty_w_hfc, 0.0f);
        np.lmw = (int)cfg_.tempogram_novelty_local_mean_window;
        np.smw = (int)cfg_.tempogram_novelty_smooth_window;
    } else {  // combined_novelty defaults (novelty.rs:868-871)
        np.ws = 0.5f;
        np.we = 0.3f;
        np.wh = 0.2f;
        np.lmw = 16;
        np.smw = 5;
    }
    np.wsum = sd_maxf(np.ws + np.we + np.wh, EPS);
    for (int v = 0; v < 4; v++) np.band_on[v] = fp.band_on[v];
    float* scratch = c_.dev<float>(tag + "novscr", 8 * std::max<uint64_t>(total, 1));
    o.nov = c_.dev<float>(tag + "nov", NVAR * std::max<uint64_t>(total, 1));
    o.nov_sum = c_.dev<float>(tag + "novsum", NVAR * (size_t)std::max(P_T, 1));
    launch_novelty(o.E, o.H, o.SFX, o.d_fpfx, P_T, total, np, scratch, o.nov, o.nov_sum, o.MEL, fp.n_mels,
                   (int)std::max<uint64_t>(cfg_.tempogram_mel_max_filter_bins, 1), mel_on,
                   c_.dev<unsigned int>(tag + "melmax", (size_t)std::max(P_T, 1)), d_.stream);
    SDSP_HIP_CHECK(hipGetLastError());
    o.nov_mr = o.nov;
    if (in.mr_nov && !band_cfg) {
        // without the auxiliary variants the tempogram's novelty uses combined_novelty's defaults,
        // but multi-resolution's hop-512 novelty still takes the configured weights
        // (multi_resolution.rs:680-694): the full-band variant again, with those
        NovParams nm = np;
        nm.ws = sd_maxf(cfg_.tempogram_novelty_w_spectral, 0.0f);
        nm.we = sd_maxf(cfg_.tempogram_novelty_w_energy, 0.0f);
        nm.wh = sd_maxf(cfg_.tempogram_novelty_w_hfc, 0.0f);
        nm.lmw = (int)cfg_.tempogram_novelty_local_mean_window;
        nm.smw = (int)cfg_.tempogram_novelty_smooth_window;
        nm.wsum = sd_maxf(nm.ws + nm.we + nm.wh, EPS);
        for (int v = 1; v < 4; v++) nm.band_on[v] = 0;
        o.nov_mr = c_.dev<float>(tag + "novmr", NVAR * std::max<uint64_t>(total, 1));
        launch_novelty(o.E, o.H, o.SFX, o.d_fpfx, P_T, total, nm, scratch, o.nov_mr,
                       c_.dev<float>(tag + "novmrsum", NVAR * (size_t)std::max(P_T, 1)), o.MEL, 0, 1, false,
                       c_.dev<unsigned int>(tag + "melmax", (size_t)std::max(P_T, 1)), d_.stream);
        SDSP_HIP_CHECK(hipGetLastError());
    }
    tm.mark(2);
    // tempograms: items (track, variant) for active tracks
    int present[NVAR];
    for (int v = 0; v < 4; v++) present[v] = fp.band_on[v];
    present[4] = mel_on;
    std::vector<int> items;
    for (int t = 0; t < P_T; t++)
        if (o.active_h[(size_t)t])
            for (int v = 0; v < NVAR; v++)
                if (present[v]) items.push_back(t * NVAR + v);
    // ACF
    std::vector<float> gb;
    std::vector<int> gl;
    acf_grid(sr_, hop, cfg_.min_bpm, cfg_.max_bpm, cfg_.bpm_resolution, &gb, &gl);
    const int NB = (int)gb.size();
    if (NB > 512) throw HipError("autocorrelation grid larger than 512 BPMs");
    float* d_gb = c_.up(tag + "acfgb", gb);
    int* d_gl = c_.up(tag + "acfgl", gl);
    int* d_items = c_.up(tag + "items", items);
    const size_t n_it = items.size();
    float* acf_bpm = c_.dev<float>(tag + "acfb", std::max<size_t>(n_it, 1) * (size_t)NB);
    float* acf_str = c_.dev<float>(tag + "acfs", std::max<size_t>(n_it, 1) * (size_t)NB);
    launch_acf_tempogram(d_items, (int)n_it, o.nov, o.d_fpfx, total, d_gb, d_gl, NB, acf_bpm, acf_str, d_.stream);
    SDSP_HIP_CHECK(hipGetLastError());
    // FFT tempograms grouped by P
    std::vector<uint64_t> fft_off(n_it, 0);
    std::vector<int> fft_k_track((size_t)P_T, 0);
    std::map<uint64_t, std::vector<int>> byP;  // P -> item positions
    for (size_t i = 0; i < n_it; i++) {
        const int t = items[i] / NVAR;
        const uint64_t L = o.fpfx[(size_t)t + 1] - o.fpfx[(size_t)t] - 1;
        byP[next_pow2(L)].push_back((int)i);
    }
    uint64_t fcur = 0;
    struct PClass {
        uint64_t P;
        FftTgParams prm;
        std::vector<int> pos;
    };
    std::vector<PClass> classes;
    for (auto& kv : byP) {
        PClass pc{kv.first, FftTgParams{}, kv.second};
        int b_lo, K;
        float fr;
        fft_bins(sr_, hop, kv.first, cfg_.min_bpm, cfg_.max_bpm, &b_lo, &K, &fr);
        pc.prm.P = (int)kv.first;
        pc.prm.b_lo = b_lo;
        pc.prm.K = K;
        pc.prm.fres = fr;
        // k_fft_tempogram's in-place LDS FFT up to P = 8192 (32 KB of LDS); larger P (3-min tracks
        // at hop 512 have P = 16384) through L2-resident global scratch.  A 64 KB LDS workgroup
        // waits for a CU that no key-stream STFT workgroup occupies, which the concurrent pipeline
        // seldom offers: its launches stretched from 0.3 ms to 19 ms (round 4)
#ifndef SDSP_FFT_TG_LDS_MAX
#define SDSP_FFT_TG_LDS_MAX 8192
#endif
        pc.prm.lds = kv.first <= SDSP_FFT_TG_LDS_MAX ? 1 : 0;
        uint64_t K2 = 1;
        while (K2 < (uint64_t)K) K2 <<= 1;
        if (K > 0 && K2 > kv.first / 2) throw HipError("FFT tempogram: too many in-range bins for the key buffer");
        for (int i : pc.pos) {
            fft_off[(size_t)i] = fcur;
            fcur += (uint64_t)K;
            fft_k_track[(size_t)(items[(size_t)i] / NVAR)] = K;
        }
        classes.push_back(pc);
    }
    float* fft_bpm = c_.dev<float>(tag + "fftb", std::max<uint64_t>(fcur, 1));
    float* fft_pow = c_.dev<float>(tag + "fftp", std::max<uint64_t>(fcur, 1));
    uint64_t* d_fft_off_items = c_.up(tag + "fftoffi", fft_off);
    for (auto& pc : classes) {
        if (pc.prm.K == 0) continue;
        std::vector<int> sub;
        std::vector<uint64_t> offs;
        for (int i : pc.pos) {
            sub.push_back(items[(size_t)i]);
            offs.push_back(fft_off[(size_t)i]);
        }
        int* d_sub = c_.up(tag + "fsub" + std::to_string(pc.P), sub);
        uint64_t* d_offs = c_.up(tag + "foff" + std::to_string(pc.P), offs);
        FftTables& ft = d_.tables((int)pc.P, false);
        cx* gscr = nullptr;
        if (!pc.prm.lds) gscr = c_.dev<cx>(tag + "fgscr", sub.size() * (size_t)pc.P);
        launch_fft_tempogram(d_sub, (int)sub.size(), P_T, o.nov, o.nov_sum, o.d_fpfx, total, pc.prm, ft.tw.as<cx>(),
                             ft.rt.as<cx>(), gscr, d_offs, fft_bpm, fft_pow, d_.stream);
        SDSP_HIP_CHECK(hipGetLastError());
    }
    (void)d_fft_off_items;
    // per (track, variant) offsets for the selector
    std::vector<uint64_t> fo((size_t)P_T * NVAR, 0), ao((size_t)P_T * NVAR, 0);
    for (size_t i = 0; i < n_it; i++) {
        fo[(size_t)items[i]] = fft_off[i];
        ao[(size_t)items[i]] = (uint64_t)i * (uint64_t)NB;
    }
    uint64_t* d_fo = c_.up(tag + "selfo", fo);
    uint64_t* d_ao = c_.up(tag + "selao", ao);
    int* d_fk = c_.up(tag + "selfk", fft_k_track);
    SelParams sp{};
    sp.min_bpm = cfg_.min_bpm;
    sp.max_bpm = cfg_.max_bpm;
    sp.ac_tol = sd_maxf(cfg_.bpm_resolution, 0.5f);
    for (int v = 0; v < NVAR; v++) sp.present[v] = present[v];
    sp.w[0] = band_cfg ? cfg_.tempogram_band_w_full : 1.0f;
    sp.w[1] = cfg_.tempogram_band_w_low;
    sp.w[2] = cfg_.tempogram_band_w_mid;
    sp.w[3] = cfg_.tempogram_band_w_high;
    sp.w[4] = cfg_.tempogram_mel_weight;
    sp.seed_only = band_cfg ? cfg_.tempogram_band_seed_only : 1;
    sp.support_thr = sd_clampf(band_cfg ? cfg_.tempogram_band_support_threshold : 0.25f, 0.0f, 1.0f);
    sp.bonus = sd_maxf(band_cfg ? cfg_.tempogram_band_consensus_bonus : 0.0f, 0.0f);
    sp.bonus_on = sp.bonus > 0.0f && band_cfg && (cfg_.enable_tempogram_band_fusion || cfg_.enable_tempogram_mel_novelty);
    sp.top_n = in.top_n;
    sp.NB = NB;
    sp.gate = in.gate;
    sp.gate_top_n = (int)std::max<uint64_t>(
        std::max<uint64_t>(cfg_.tempogram_candidates_top_n, cfg_.tempogram_multi_res_top_k), 10);
    sp.gate_tol = sd_maxf(2.0f, cfg_.bpm_resolution);
    o.est = c_.dev<TempoEst>(tag + "est", (size_t)std::max(P_T, 1));
    o.cand = c_.dev<float>(tag + "cand", (size_t)std::max(P_T, 1) * (size_t)in.cand_cap * 4);
    launch_tempo_select(P_T, o.active, fft_bpm, fft_pow, d_fo, d_fk, acf_bpm, acf_str, d_ao, sp, o.est, o.cand,
                               in.cand_cap, d_.stream);
    SDSP_HIP_CHECK(hipGetLastError());
    tm.mark(3);
    c_.sync();
    o.stft_ms = tm.ms(0, 1);
    o.feat_ms = tm.ms(1, 2);
    o.tempo_ms = tm.ms(2, 3);
}

}  // namespace sdsp

namespace sdsp {

// SDSP_HOST_TRACE=1: host wall time between the sub-batch's synchronisation points (stderr)
std::vector<size_t> Pipeline::finish_key(std::vector<TrackRes>& res, bool keep_tail) {
    std::vector<size_t> near;
    if (!key_pending_) return near;
    std::unique_ptr<KeyPending> kp = std::move(key_pending_);
    SDSP_HIP_CHECK(hipStreamWaitEvent(d_.stream, kp->kt->ev[2], 0));
    const std::vector<KeyOut> kout = c_.down(kp->d_kout, kp->at.size());
    for (size_t k = 0; k < kp->at.size(); k++) {
        TrackRes& r = res[kp->at[k]];
        const KeyOut& ko = kout[k];
        if (!ko.ok) continue;
        r.key_mode = ko.mode;
        r.key_tonic = ko.tonic;
        r.key_conf = ko.conf;
        r.key_clarity = ko.clarity;
        r.key_near = ko.near;
        if (ko.near) near.push_back(kp->at[k]);
    }
    times_.stft8192_ms += kp->kt->ms(0, 1);
    times_.key_ms += kp->kt->ms(1, 2);
    if (keep_tail && kp->tail.ok) tail_ = std::move(kp);
    return near;
}

// The exact key rerun of the call's last sub-batch's near-decision tracks, in place:
// the reference's sequential frame-energy fold needs every masked bin, and the band path stored only
// HPCP's band.  The bins outside it still hold the STFT's magnitudes, so k_mask_rp completes the
// masked spectrogram there (the same masked values the nested rerun's full-bin mask stores), k_hpcp
// folds each frame's energy in bin order (and rewrites the same chroma), and the vote runs on the
// exact energies: the nested rerun's results without its front end and 8192-point STFT.
void Pipeline::rerun_tail(const std::vector<size_t>& near, std::vector<TrackRes>& res) {
    std::unique_ptr<KeyPending> kp = std::move(tail_);
    if (near.empty() || !kp || exact_energy_ || nested_) return;
    const KeyTail& t = kp->tail;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<int> sel;
    for (size_t i : near)
        for (size_t k = 0; k < kp->at.size(); k++)
            if (kp->at[k] == i) sel.push_back((int)k);
    if (sel.size() != near.size()) throw HipError("rerun_tail: a near track is not in the last sub-batch");
    const int n = (int)sel.size();
    std::vector<uint64_t> tp(1, 0), sp(1, 0);
    for (int k : sel) {
        const uint64_t F = t.kpfx[(size_t)k + 1] - t.kpfx[(size_t)k];
        tp.push_back(tp.back() + (F + HP_FRAMES - 1) / HP_FRAMES);
        sp.push_back(sp.back() + (t.kseg[(size_t)k + 1] - t.kseg[(size_t)k]));
    }
    hipStream_t st = d_.stream;
    int* d_sel = c_.up("E.tail_sel", sel);
    uint64_t* d_tp = c_.up("E.tail_tile", tp);
    uint64_t* d_sp = c_.up("E.tail_seg", sp);
    launch_mask_band(t.mags8, ks_, t.B8, t.d_kpfx, d_sel, n, cfg_.key_harmonic_mask_power, t.st_lo, t.st_hi, t.d_part,
                     t.total8, st, true);
    SDSP_HIP_CHECK(hipGetLastError());
    launch_hpcp(t.mags8, t.d_kpfx, d_tp, d_sel, n, tp.back(), t.hp, t.d_ht, t.d_chroma, t.d_energy, st);
    SDSP_HIP_CHECK(hipGetLastError());
    KeyParams kx = t.kp;
    kx.near_check = 0;  // the exact energies: nothing left to certify
    // (the vote writes out[track], so the selected tracks' entries of the sub-batch's KeyOut array)
    launch_key_vote(d_sel, n, t.d_kpfx, t.d_chroma, t.d_energy, t.d_cs, t.d_w, t.d_sscr, d_sp, t.d_tpl, kx, kp->d_kout,
                    st, nullptr, nullptr, nullptr, true);
    SDSP_HIP_CHECK(hipGetLastError());
    const std::vector<KeyOut> ko = c_.down(kp->d_kout, kp->at.size());
    for (int j = 0; j < n; j++) {
        TrackRes& r = res[near[(size_t)j]];
        const KeyOut& o = ko[(size_t)sel[(size_t)j]];
        if (!o.ok) {
            r.status = SDSP_ERR_PROCESSING;
            r.err = "Processing error: key certification rerun failed (no key from the exact energies)";
            continue;
        }
        r.key_mode = o.mode;
        r.key_tonic = o.tonic;
        r.key_conf = o.conf;
        r.key_clarity = o.clarity;
        r.key_rerun = true;
    }
    reruns_ += (uint64_t)n;
    rerun_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// The exact key rerun of near-decision tracks for a finished sub-batch, from inside
// the main pass: a nested key-only pipeline with the sequential energy fold, its buffers prefixed
// ("X.") and its key path on the main stream, whose queue then runs it in the slack the tempo path
// leaves beside the key stream.  The tracks of the last sub-batch are rerun by run_locked.
void Pipeline::rerun_near(const float* d_samples, const std::vector<uint64_t>& in_off, const std::vector<uint64_t>& n_raw,
                          const std::vector<size_t>& near, std::vector<TrackRes>& res) {
    if (near.empty() || exact_energy_ || nested_) return;
    std::vector<uint64_t> o2, l2;
    for (size_t i : near) o2.push_back(in_off[i]), l2.push_back(n_raw[i]);
    std::vector<TrackRes> r2;
    Pipeline px(d_, cfg_, sr_, SDSP_STAGES_FULL, true, true, true);
    px.run(d_samples, o2, l2, r2);
    for (size_t j = 0; j < near.size(); j++) {
        TrackRes& r = res[near[j]];
        if (r2[j].status != SDSP_OK) {  // the key fields are not certified: the track fails
            r.status = SDSP_ERR_PROCESSING;
            r.err = "Processing error: key certification rerun failed (" + r2[j].err + ")";
            continue;
        }
        r.key_mode = r2[j].key_mode;
        r.key_tonic = r2[j].key_tonic;
        r.key_conf = r2[j].key_conf;
        r.key_clarity = r2[j].key_clarity;
        r.key_rerun = true;
    }
    reruns_ += near.size();
    rerun_ms_ += d_.last.total_ms;  // px.run's
}

struct HostTrace {
    bool on = test_hooks().host_trace.load() != 0;  // sdsp_debug_set_schedule
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), tp = t0;
    void operator()(const char* tag) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[sdsp host] %-12s +%8.3f ms  (%8.3f)\n", tag,
                     std::chrono::duration<double, std::milli>(t - tp).count(),
                     std::chrono::duration<double, std::milli>(t - t0).count());
        tp = t;
    }
};

void Pipeline::sub_batch(const float* d_samples, const std::vector<uint64_t>& in_off, const std::vector<uint64_t>& n_raw,
                         const std::vector<int>& idx, std::vector<TrackRes>& res) {
    const int T = (int)idx.size();
    const int FS = fs_;
    const int HOP = (int)cfg_.hop_size;
    hipStream_t st = d_.stream;
    HostTrace htr;
    Timers tm;
    tm.init(d_);
    tm.mark(0);
    // ---------------- A: peak/gain, silence, trim ----------------
    std::vector<uint64_t> off((size_t)T), nr((size_t)T), cpfx((size_t)T + 1, 0), spfx((size_t)T + 1, 0);
    for (int t = 0; t < T; t++) {
        off[(size_t)t] = in_off[(size_t)idx[(size_t)t]];
        nr[(size_t)t] = n_raw[(size_t)idx[(size_t)t]];
        cpfx[(size_t)t + 1] = cpfx[(size_t)t] + (nr[(size_t)t] + PK_CH - 1) / PK_CH;
        const uint64_t fs = nr[(size_t)t] >= (uint64_t)FS ? (nr[(size_t)t] - FS) / (FS / 2) + 1 : 1;
        spfx[(size_t)t + 1] = spfx[(size_t)t] + (cfg_.enable_silence_trimming ? fs : 0);
    }
    uint64_t* d_off = c_.up("A.off", off);
    uint64_t* d_nr = c_.up("A.nr", nr);
    uint64_t* d_cpfx = c_.up("A.cpfx", cpfx);
    uint64_t* d_spfx = c_.up("A.spfx", spfx);
    unsigned int* d_peak = c_.dev<unsigned int>("A.peak", (size_t)T);
    float* d_gain = c_.dev<float>("A.gain", (size_t)T);
    const float target = sd_powf(10.0f, (0.0f - 1.0f) / 20.0f);  // lib.rs:121 max_headroom_db = 1.0
    const bool loud = cfg_.enable_normalization && cfg_.normalization != SDSP_NORM_PEAK;
    std::vector<int> nstat((size_t)T, 0);
    if (loud) {  // gains from the batch-wide pre-pass (loudness_prepass)
        std::vector<float> g((size_t)T);
        for (int t = 0; t < T; t++) {
            g[(size_t)t] = loud_gain_[(size_t)idx[(size_t)t]];
            nstat[(size_t)t] = loud_stat_[(size_t)idx[(size_t)t]];
        }
        d_gain = c_.up("A.gain", g);
    } else {
        launch_peak_gain(d_samples, d_off, d_nr, d_cpfx, T, cpfx[(size_t)T],
                         c_.dev<unsigned int>("A.peakchunk", std::max<uint64_t>(cpfx[(size_t)T], 1)), d_peak, target,
                         cfg_.enable_normalization, d_gain, st);
    }
    // One read of the samples for both frame-RMS passes: with trimming on and the trim hop (fs / 2)
    // a multiple of the energy hop, the trim pass runs on the raw signal at the energy hop (trim
    // frame f = raw frame f * (fs / 2) / hop), and the energy pass takes its whole frames from it
    // (launch_frame_rms_from_raw)
    const int G_e = HOP > 0 && FS % HOP == 0 ? FS / HOP : 0;
    const bool rms_shared = cfg_.enable_silence_trimming && HOP > 0 && HOP % 32 == 0 && (FS / 2) % HOP == 0 &&
                            (G_e == 1 || G_e == 2 || G_e == 4 || G_e == 8);
    std::vector<uint64_t> rpfx((size_t)T + 1, 0);
    for (int t = 0; t < T; t++)
        rpfx[(size_t)t + 1] = rpfx[(size_t)t] + (rms_shared ? (nr[(size_t)t] >= (uint64_t)FS ? (nr[(size_t)t] - FS) / HOP + 1 : 1) : 0);
    float* d_srms = nullptr;
    uint64_t* d_rpfx = nullptr;
    if (rms_shared) {
        d_rpfx = c_.up("A.rpfx", rpfx);
        d_srms = c_.dev<float>("A.rrms", std::max<uint64_t>(rpfx[(size_t)T], 1));
        launch_frame_rms(d_samples, d_off, d_gain, d_nr, d_rpfx, T, rpfx[(size_t)T], FS, HOP, d_srms, st);
    } else {
        d_srms = c_.dev<float>("A.srms", spfx[(size_t)T]);
        launch_frame_rms(d_samples, d_off, d_gain, d_nr, d_spfx, T, spfx[(size_t)T], FS, FS / 2, d_srms, st);
    }
    const float thr = sd_powf(10.0f, cfg_.min_amplitude_db / 20.0f);
    const uint64_t min_samples = sd_f2u64((float)500u / 1000.0f * (float)sr_);
    const uint64_t min_frames = (min_samples + (FS / 2) - 1) / (FS / 2);
    uint64_t* d_ts = c_.dev<uint64_t>("A.ts", (size_t)T);
    uint64_t* d_te = c_.dev<uint64_t>("A.te", (size_t)T);
    launch_trim(d_srms, d_spfx, T, d_nr, FS / 2, thr, min_frames, cfg_.enable_silence_trimming, d_ts, d_te, st,
                rms_shared ? d_rpfx : nullptr, rms_shared ? (FS / 2) / HOP : 1);
    SDSP_HIP_CHECK(hipGetLastError());
    std::vector<float> gain_h = c_.down(d_gain, (size_t)T);
    std::vector<uint64_t> ts = c_.down(d_ts, (size_t)T), te = c_.down(d_te, (size_t)T);
    htr("A");
    tm.mark(1);
    // remaining tracks (non-empty after trimming)
    std::vector<int> R;  // positions in idx
    for (int t = 0; t < T; t++) {
        TrackRes& r = res[(size_t)idx[(size_t)t]];
        const uint64_t n = te[(size_t)t] - ts[(size_t)t];
        if (nstat[(size_t)t] != 0) {
            r.status = SDSP_ERR_NUMERICAL;
            r.err = "Numerical error: Mean square too small for LUFS calculation";
            continue;
        }
        if (n == 0) {
            r.status = SDSP_ERR_PROCESSING;
            r.err = "Processing error: Audio is entirely silent after trimming";
            continue;
        }
        r.duration = (float)n / (float)sr_;
        R.push_back(t);
    }
    const int NR = (int)R.size();
    if (NR == 0) return;
    const bool dbg_on = cfg_.has_debug_track_id != 0;  // debug_track_id dumps (print_debug)
    std::vector<TrackDbg> tdbg(dbg_on ? (size_t)NR : 0);
    // ---------------- B: base tempo pass (hop = config hop) + onsets ----------------
    // force_legacy_bpm skips the tempogram estimate (src/lib.rs:337): no escalation, no
    // candidates, the flags stay None; the hop-512 pass still feeds the onset detectors
    const bool tg_on = !cfg_.force_legacy_bpm;
    const bool mr_on = cfg_.enable_tempogram_multi_resolution && tg_on;
    const int base_top_n =
        (int)std::max<uint64_t>(std::max<uint64_t>(cfg_.tempogram_candidates_top_n, cfg_.tempogram_multi_res_top_k), 10);
    TempoPassIn bin;
    bin.hop = HOP;
    bin.samples = d_samples;
    for (int t : R) {
        bin.src_off.push_back(off[(size_t)t] + ts[(size_t)t]);
        bin.gain_h.push_back(gain_h[(size_t)t]);
        bin.n_trim.push_back(te[(size_t)t] - ts[(size_t)t]);
    }
    bin.want_onsets = true;
    bin.top_n = mr_on ? base_top_n : (cfg_.emit_tempogram_candidates ? (int)cfg_.tempogram_candidates_top_n : 1);
    bin.cand_cap = std::max(bin.top_n, 1);
    bin.gate = mr_on;
    bin.mr_nov = mr_on && HOP == 512;  // at another hop the escalation runs its own hop-512 pass
    // ---------------- E: key (second stream; overlaps B-D) ----------------
    // The key path depends only on the trimmed signal, so it is forked onto the context's key
    // stream right after trimming and joined before the results are read back: its
    // bandwidth-bound STFT/mask/HPCP kernels run under the latency-bound tempo and beat
    // kernels of the main stream.
    const int KFS = kfs_, KHOP = khop_;
    std::vector<int> K;  // positions in R
    std::vector<uint64_t> kpfx(1, 0), ktile(1, 0), kseg(1, 0), ksrc;
    std::vector<float> kgain;
    const int seg_len_cfg = (int)std::min<uint64_t>(cfg_.key_segment_len_frames, INT32_MAX);
    const int seg_hop = (int)std::max<uint64_t>(std::min<uint64_t>(cfg_.key_segment_hop_frames, (uint64_t)seg_len_cfg), 1);
    const bool seg_voting = cfg_.enable_key_segment_voting && cfg_.key_segment_len_frames >= 120 &&
                            cfg_.key_segment_hop_frames >= 1;
    const bool ms_on = cfg_.enable_key_multi_scale && cfg_.key_multi_scale_lengths_len > 0;
    const uint64_t ms_hop = std::max<uint64_t>(std::min<uint64_t>(cfg_.key_multi_scale_hop, INT32_MAX), 1);
    // segment scratch rows of a chroma slice of F rows (an upper bound: edge trim only shortens it)
    auto seg_rows = [&](uint64_t F) -> uint64_t {
        uint64_t ns = (seg_voting && F >= (uint64_t)std::max(seg_len_cfg, 1)) ? (F - seg_len_cfg) / seg_hop + 1 : 0;
        if (ms_on) {
            uint64_t nm = 0;
            for (uint64_t j = 0; j < cfg_.key_multi_scale_lengths_len; j++) {
                const uint64_t len = cfg_.key_multi_scale_lengths[j];
                if (len != 0 && len <= F) nm += (F - len) / ms_hop + 1;
            }
            ns = std::max(ns, nm);
        }
        return ns;
    };
    double key_in_bytes = 0;
    for (int i = 0; i < NR; i++) {
        const uint64_t n = bin.n_trim[(size_t)i];
        if (bpm_only_) break;  // SDSP_STAGES_BPM_ONLY: stages a1-a19 only, no key path
        if (n < (uint64_t)FS || n < (uint64_t)KFS) continue;  // key skipped or empty key spectrogram -> default key
        const uint64_t F8 = (n - KFS) / (uint64_t)KHOP + 1;
        K.push_back(i);
        kpfx.push_back(kpfx.back() + F8);
        ktile.push_back(ktile.back() + (F8 + HP_FRAMES - 1) / HP_FRAMES);
        kseg.push_back(kseg.back() + (uint64_t)KV_ROW * seg_rows(F8));
        ksrc.push_back(bin.src_off[(size_t)i]);
        kgain.push_back(bin.gain_h[(size_t)i]);
        key_in_bytes += 4.0 * (double)n;
    }
    const int NK = (int)K.size();
    std::vector<KeyOut> kout;
    KeyOut* d_kout = nullptr;
    KeyDbg* d_kdbg = nullptr;
    std::unique_ptr<Timers> ktp(new Timers());
    Timers& kt = *ktp;
    kt.init(d_);
    // what the main stream uploads for the key stream (read by it before the sub-batch's join)
    sb_parity_ ^= 1;
    const std::string EP = sb_parity_ ? "E1." : "E0.";
    // schedule knob (sdsp_debug_set_schedule): the key path on the main stream (per-kernel profiling)
    const bool serial_streams = nested_ || test_hooks().serial_streams.load() != 0;
    hipStream_t st2 = serial_streams ? st : d_.stream2;
    hipStream_t st3 = serial_streams ? st : d_.stream3;  // the key vote
    float* d_tune = nullptr;  // per key track tuning offset (tuning compensation)
    float* mags8 = nullptr;
    uint64_t* d_kpfx = nullptr;
    uint64_t* d_ktile = nullptr;
    int* d_kid = nullptr;
    float* d_tpl = nullptr;
    KeyParams kp{};
    KeyTail ktail;  // the band path's state for rerun_tail
    const int B8 = KFS / 2 + 1;
    const float fres8 = (float)sr_ / (float)KFS;
    if (NK > 0) {
        const uint64_t total8 = kpfx.back();
        d_kpfx = c_.up(EP + "kpfx", kpfx);
        d_ktile = c_.up(EP + "ktile", ktile);
        uint64_t* d_kseg = c_.up(EP + "kseg", kseg);
        const std::vector<uint64_t> kstr = stft_strips(kpfx);
        uint64_t* d_kstr = c_.up(EP + "kstrip", kstr);
        uint64_t* d_ksrc = c_.up(EP + "ksrc", ksrc);
        float* d_kgain = c_.up(EP + "kgain", kgain);
        std::vector<int> kid((size_t)NK);
        for (int k = 0; k < NK; k++) kid[(size_t)k] = k;
        d_kid = c_.up(EP + "kid", kid);
        FftTables& t8 = d_.tables(KFS, true);
        mags8 = c_.dev<float>("E.mags8", total8 * ks_);
        // uploads above were queued on the main stream: order the key stream after them
        kt.mark(7);
        SDSP_HIP_CHECK(hipStreamWaitEvent(st2, kt.ev[7], 0));
        kt.mark(0, st2);
        launch_stft(KFS, false, d_samples, d_kpfx, NK, total8, d_ksrc, d_kgain, KHOP, t8.window.as<float>(),
                    stft_twp(t8, KFS, false), stft_rtp(t8, KFS, false), mags8, d_kpfx, ks_, nullptr, st2, d_kstr, kstr.back(),
                    c_.dev<uint32_t>("E.redo", total8 + 1));
        SDSP_HIP_CHECK(hipGetLastError());
        kt.mark(1, st2);
        // key spectrogram conditioning (src/lib.rs:1011-1060): the mask runs in place over HBM
        // (k_mask_r), then HPCP reads the masked spectrogram (DESIGN.md §4 on the fused variant)
        const bool use_log = cfg_.enable_key_log_frequency;  // :1062-1095
        const bool tuned = cfg_.enable_key_tuning_compensation && !use_log;
        const bool whiten = cfg_.enable_key_hpcp_whitening && cfg_.key_hpcp_whitening_smooth_bins >= 3;
        // the default key path (harmonic mask, plain HPCP, nothing else reading the masked
        // spectrogram): the mask stores only HPCP's peak band and folds the frame energies in
        // 64-bin blocks (k_mask_rp / k_hpcp_band); SDSP_KEY_EXACT_ENERGY builds
        // keep the reference's one sequential energy sum (k_mask_r / k_hpcp)
        HpcpParams hp{};
        hp.B = B8;
        hp.stride = ks_;
        key_peak_band(cfg_, sr_, &hp.pk_lo, &hp.pk_hi);
        hp.K = (int)std::max<uint64_t>(cfg_.key_hpcp_peaks_per_frame, 1);
        hp.hmax = (int)std::max<uint64_t>(cfg_.key_hpcp_num_harmonics, 1);
        hp.p = sd_clampf(cfg_.key_hpcp_mag_power, 0.05f, 1.0f);
        // sdsp_debug_key_energy_blocked answers the same; exact_energy_: the rerun of near-decision tracks
        // exact_energy_ on the same configurations (the rerun): the band path's mask storing every
        // bin (its masked values are k_mask_r's, bit for bit, at less cost), then k_hpcp's one
        // sequential energy sum; the block sums it also writes go unused
        const bool blocked = key_energy_blocked(cfg_, sr_);
        const bool band = blocked && !exact_energy_;
        float* d_part = blocked ? c_.dev<float>("E.kpart", total8 * (uint64_t)((B8 + 63) / 64)) : nullptr;
        if (blocked) {
            launch_mask_band(mags8, ks_, B8, d_kpfx, d_kid, NK, cfg_.key_harmonic_mask_power, band ? hp.pk_lo - 1 : 0,
                             band ? hp.pk_hi + 1 : B8 - 1, d_part, total8, st2);
        } else if (cfg_.enable_key_hpss_harmonic) {
            const KeyHpssParams kh = key_hpss_params(cfg_, sr_, B8, fres8, ks_);
            if (kh.nb > 0) {  // an empty band returns the spectrogram unchanged (extractor.rs:1408-1410)
                std::vector<uint64_t> moff(1, 0), mt(1, 0), at(1, 0);
                for (int k = 0; k < NK; k++) {
                    const uint64_t F8 = kpfx[(size_t)k + 1] - kpfx[(size_t)k];
                    const uint64_t nds = (F8 + (uint64_t)kh.step - 1) / (uint64_t)kh.step;
                    moff.push_back(moff.back() + nds * (uint64_t)kh.nb);
                    mt.push_back(mt.back() + ((nds + KH_TILE_FRAMES - 1) / KH_TILE_FRAMES) *
                                                 (((uint64_t)kh.nb + KH_TILE_BINS - 1) / KH_TILE_BINS));
                    at.push_back(at.back() + (F8 + KH_APPLY_FRAMES - 1) / KH_APPLY_FRAMES);
                }
                uint64_t* d_moff = c_.up(EP + "kh_off", moff);
                uint64_t* d_mt = c_.up(EP + "kh_mt", mt);
                uint64_t* d_at = c_.up(EP + "kh_at", at);
                float* d_kmask = c_.dev<float>("E.kh_mask", std::max<uint64_t>(moff.back(), 1));
                // the uploads are on the main stream
                kt.mark(9);
                SDSP_HIP_CHECK(hipStreamWaitEvent(st2, kt.ev[9], 0));
                launch_key_hpss(mags8, d_kpfx, d_mt, mt.back(), d_at, at.back(), d_moff, d_kid, NK, kh, d_kmask, st2);
            }
        } else if (cfg_.enable_key_harmonic_mask)
            launch_mask(mags8, ks_, B8, d_kpfx, d_kid, NK, (int)cfg_.key_spectrogram_smooth_margin,
                        cfg_.key_harmonic_mask_power, st2);
        else if (cfg_.enable_key_spectrogram_time_smoothing)
            launch_mask(mags8, ks_, B8, d_kpfx, d_kid, NK, (int)cfg_.key_spectrogram_smooth_margin,
                        cfg_.key_harmonic_mask_power, st2, true);
        // tuning offset per track (:1097-1119)
        if (tuned) {
            TuningParams tp = tuning_params(cfg_, sr_, B8, fres8, ks_);
            d_tune = c_.dev<float>("E.tune", (size_t)NK);
            launch_tuning(mags8, d_kpfx, d_kid, NK, tp, d_tune, st2);
            SDSP_HIP_CHECK(hipGetLastError());
        }
        float* d_chroma = c_.dev<float>("E.chroma", total8 * 12);
        float* d_energy = c_.dev<float>("E.energy", total8);
        float* d_edel = nullptr;  // the band path's per-frame energy bounds (the vote's certificate)
        // the previous sub-batch's key vote (stream3) reads E.chroma / E.energy: the producers
        // below wait for it (an event never recorded counts as complete)
        // (a nested rerun has its own "X." buffers and runs in order on the main stream)
        if (!nested_) SDSP_HIP_CHECK(hipStreamWaitEvent(st2, d_.vote_done, 0));
        if (use_log) {  // :1120-1131
            const ChromaParams cp = chroma_params(cfg_, sr_, 1, B8, fres8, ks_);
            launch_chroma(1, mags8, d_kpfx, d_ktile, d_kid, NK, ktile.back(), cp, nullptr, d_chroma, d_energy, st2);
        } else if (cfg_.enable_key_hpcp && (d_tune || whiten || cfg_.enable_key_hpcp_bass_blend)) {  // :1133-1168
            const HpcpXParams hx = hpcp_x_params(cfg_, sr_, B8, fres8, whiten, ks_);
            launch_hpcp_x(mags8, d_kpfx, d_ktile, d_kid, NK, ktile.back(), hx, d_tune, d_chroma, d_energy, st2);
        } else if (cfg_.enable_key_hpcp) {
            std::vector<HarmEntry> ht =
                harm_table(B8, sr_, KFS, cfg_.soft_mapping_sigma, hp.hmax, cfg_.key_hpcp_harmonic_decay);
            HarmEntry* d_ht = c_.up(EP + "harm", ht);
            ktail.d_ht = d_ht;
            // the table upload is queued on the main stream: order the key stream after it
            kt.mark(10);
            SDSP_HIP_CHECK(hipStreamWaitEvent(st2, kt.ev[10], 0));
            if (band) {
                d_edel = c_.dev<float>("E.edel", total8);
                launch_hpcp_band(mags8, d_kpfx, d_ktile, d_kid, NK, ktile.back(), hp, d_ht, d_part, total8, d_chroma,
                                 d_energy, d_edel, st2);
            }
            else
                launch_hpcp(mags8, d_kpfx, d_ktile, d_kid, NK, ktile.back(), hp, d_ht, d_chroma, d_energy, st2);
        } else {  // :1169-1197 (the tuned variant only when |offset| > 1e-6)
            const ChromaParams cp = chroma_params(cfg_, sr_, 0, B8, fres8, ks_);
            launch_chroma(0, mags8, d_kpfx, d_ktile, d_kid, NK, ktile.back(), cp, d_tune, d_chroma, d_energy, st2);
        }
        SDSP_HIP_CHECK(hipGetLastError());
        std::vector<float> tpl(576);
        key_templates(tpl.data());
        d_tpl = c_.up(EP + "tpl", tpl);
        kp.near_check = band ? 1 : 0;
        kp.cert_fixed = test_hooks().key_cert_fixed.load();  // sdsp_debug_set_key_cert
        kp.weighting = cfg_.enable_key_frame_weighting;
        kp.min_tonal = cfg_.key_min_tonalness;
        kp.tonal_pow = cfg_.key_tonalness_power;
        kp.energy_pow = cfg_.key_energy_power;
        kp.seg_voting = seg_voting;
        kp.seg_len = std::max(seg_len_cfg, 1);
        kp.seg_hop = seg_hop;
        kp.min_clarity = sd_clampf(cfg_.key_segment_min_clarity, 0.0f, 1.0f);
        kp.sharpen = cfg_.chroma_sharpening_power;
        kp.edge_trim = cfg_.enable_key_edge_trim;
        kp.edge_frac = cfg_.key_edge_trim_fraction;
        kp.ensemble = cfg_.enable_key_ensemble;
        kp.kk_w = cfg_.key_ensemble_kk_weight;
        kp.tp_w = cfg_.key_ensemble_temperley_weight;
        kp.tset = cfg_.key_template_set == SDSP_TEMPLATES_TEMPERLEY ? 1 : 0;
        kp.mh_on = cfg_.enable_key_mode_heuristic || cfg_.enable_key_minor_harmonic_bonus;
        kp.mh_bonus = cfg_.enable_key_minor_harmonic_bonus;
        kp.mh_margin = cfg_.key_mode_third_ratio_margin;
        kp.mh_flip = cfg_.enable_key_mode_heuristic ? cfg_.key_mode_flip_min_score_ratio : 0.0f;
        kp.mh_bonus_w = cfg_.key_minor_leading_tone_bonus_weight;
        kp.ms_on = ms_on;
        kp.ms_n = ms_on ? (int)cfg_.key_multi_scale_lengths_len : 0;
        kp.ms_hop = (int)ms_hop;
        kp.ms_nw = (int)std::min<uint64_t>(cfg_.key_multi_scale_weights_len, 8);
        kp.ms_min_cl = sd_clampf(cfg_.key_multi_scale_min_clarity, 0.0f, 1.0f);
        for (int j = 0; j < kp.ms_n; j++)
            kp.ms_len[j] = (int)std::min<uint64_t>(cfg_.key_multi_scale_lengths[j], INT32_MAX);
        for (int j = 0; j < kp.ms_nw; j++) kp.ms_w[j] = cfg_.key_multi_scale_weights[j];
        float* d_cs = c_.dev<float>("E.chroma_s", total8 * 12);
        float* d_w = c_.dev<float>("E.weights", total8);
        float* d_sscr = c_.dev<float>("E.segscr", std::max<uint64_t>(kseg.back(), 1));
        d_kout = c_.dev<KeyOut>(EP + "kout", (size_t)NK);
        if (band && ktail.d_ht) {
            ktail.ok = true;
            ktail.mags8 = mags8;
            ktail.d_kpfx = d_kpfx;
            ktail.kpfx = kpfx;
            ktail.kseg = kseg;
            ktail.d_part = d_part;
            ktail.total8 = total8;
            ktail.st_lo = hp.pk_lo - 1;
            ktail.st_hi = hp.pk_hi + 1;
            ktail.B8 = B8;
            ktail.hp = hp;
            ktail.d_chroma = d_chroma;
            ktail.d_energy = d_energy;
            ktail.d_cs = d_cs;
            ktail.d_w = d_w;
            ktail.d_sscr = d_sscr;
            ktail.d_tpl = d_tpl;
        }
        // the template upload above is on the main stream too; the vote follows the chroma on st2
        kt.mark(8);
        kt.mark(11, st2);
        SDSP_HIP_CHECK(hipStreamWaitEvent(st3, kt.ev[8], 0));
        SDSP_HIP_CHECK(hipStreamWaitEvent(st3, kt.ev[11], 0));
        d_kdbg = dbg_on ? c_.dev<KeyDbg>(EP + "kdbg", (size_t)NK) : nullptr;
        float* d_wdel = d_edel ? c_.dev<float>("E.wdel", total8) : nullptr;
        // the call's last sub-batch votes with nothing beside it on the chip (its tail)
        launch_key_vote(d_kid, NK, d_kpfx, d_chroma, d_energy, d_cs, d_w, d_sscr, d_kseg, d_tpl, kp, d_kout, st3, d_kdbg,
                        d_edel, d_wdel, last_sub_ || nested_ || key_only_);
        SDSP_HIP_CHECK(hipGetLastError());
        kt.mark(2, st3);
        if (!nested_) SDSP_HIP_CHECK(hipEventRecord(d_.vote_done, st3));
        times_.stft8192_launches += 1;
        times_.stft8192_frames += total8;
        times_.stft8192_bytes += key_in_bytes + 4.0 * (double)total8 * (double)B8;
    }
    if (key_only_) {  // run_locked's exact key rerun: the key fields only (the tempo path is not run)
        if (NK > 0) {
            SDSP_HIP_CHECK(hipStreamWaitEvent(st, kt.ev[2], 0));
            const std::vector<KeyOut> ko = c_.down(d_kout, (size_t)NK);
            for (int k = 0; k < NK; k++) {
                TrackRes& r = res[(size_t)idx[(size_t)R[(size_t)K[(size_t)k]]]];
                if (!ko[(size_t)k].ok) continue;
                r.key_mode = ko[(size_t)k].mode;
                r.key_tonic = ko[(size_t)k].tonic;
                r.key_conf = ko[(size_t)k].conf;
                r.key_clarity = ko[(size_t)k].clarity;
            }
        }
        htr("E key only");
        return;
    }
    TempoPassOut bo;
    tempo_pass("B.", bin, bo);
    times_.stft2048_ms += bo.stft_ms;
    times_.stft2048_launches += bo.stft_launch;
    times_.stft2048_frames += bo.stft_frames;
    times_.stft2048_bytes += bo.stft_bytes;
    times_.features_ms += bo.feat_ms;
    times_.tempogram_ms += bo.tempo_ms;
    tm.mark(2);
    // HPSS (hpss.rs:71-172) of the hop-512 spectrogram: for the HPSS onsets every track
    // (src/lib.rs:222-236), for the percussive tempogram fallback only the tracks in the low
    // trap zone (src/lib.rs:587-598); both read the same decomposition.
    const bool hpss_on = cfg_.enable_hpss_onsets && cfg_.enable_onset_consensus;
    const bool perc_on = mr_on && cfg_.enable_tempogram_percussive_fallback;
    std::vector<TempoEst> best;
    std::vector<int> S;                 // HPSS items (positions in R)
    std::vector<uint64_t> hpfx(1, 0);   // frame prefix over S
    float *d_P0 = nullptr, *d_hpe = nullptr, *d_hfmax = nullptr;
    if (hpss_on || perc_on) {
        best = c_.down(bo.est, (size_t)NR);
        for (int i = 0; i < NR; i++) {
            const TempoEst& e = best[(size_t)i];
            if (hpss_on || (e.ok && e.ambiguous && e.trap_low)) {
                S.push_back(i);
                hpfx.push_back(hpfx.back() + (bo.fpfx[(size_t)i + 1] - bo.fpfx[(size_t)i]));
            }
        }
        const int NS = (int)S.size();
        const uint64_t totS = hpfx.back();
        if (NS > 0 && totS > 0) {
            std::vector<uint64_t> orow, vt(1, 0), rt(1, 0);
            const uint64_t ncb = (nb_ + HPSS_COLS - 1) / HPSS_COLS;
            for (int k = 0; k < NS; k++) {
                const uint64_t F = hpfx[(size_t)k + 1] - hpfx[(size_t)k];
                orow.push_back(bo.fpfx[(size_t)S[(size_t)k]]);
                vt.push_back(vt.back() + (F + HPSS_VM_FRAMES - 1) / HPSS_VM_FRAMES * ncb);
                rt.push_back(rt.back() + (F + HPSS_ROW_FRAMES - 1) / HPSS_ROW_FRAMES);
            }
            HpssLaunch L{};
            L.P.B = nb_;
            L.P.stride = s2_;
            L.P.m = (int)cfg_.hpss_margin;
            L.orig = bo.mags;
            L.orig_row0 = c_.up("H.orow", orow);
            for (int q = 0; q < 2; q++) {
                L.h[q] = c_.dev<float>("H.h" + std::to_string(q), totS * s2_);
                L.p[q] = c_.dev<float>("H.p" + std::to_string(q), totS * s2_);
            }
            uint64_t* d_hpfx = c_.up("H.hpfx", hpfx);
            L.row0 = d_hpfx;
            L.fpfx = d_hpfx;
            L.vtile_pfx = c_.up("H.vt", vt);
            L.n_vtiles = vt.back();
            L.last_it = c_.up("H.last", std::vector<int>((size_t)NS, 9));
            L.change = c_.dev<unsigned int>("H.chg", (size_t)NS);
            L.n_items = NS;
            launch_hpss(L, st);
            SDSP_HIP_CHECK(hipGetLastError());
            d_P0 = L.p[0];
            d_hpe = c_.dev<float>("H.e", totS);
            d_hfmax = c_.dev<float>("H.fmax", totS);
            launch_hpss_rows(d_P0, d_hpfx, d_hpfx, c_.up("H.rt", rt), rt.back(), NS, s2_, nb_, d_hpe, d_hfmax, st);
            SDSP_HIP_CHECK(hipGetLastError());
            htr("HPSS");
        }
    }
    // onsets: energy flux (frame FS, hop HOP; same framing as the STFT), spectral flux, HFC, HPSS, consensus
    uint64_t* d_src = c_.up("B.src2", bin.src_off);
    float* d_g = c_.up("B.gain2", bin.gain_h);
    uint64_t* d_nt = c_.up("B.ntrim", bin.n_trim);
    float* d_erms = c_.dev<float>("B.erms", std::max<uint64_t>(bo.total, 1));
    bool from_raw = rms_shared;
    std::vector<uint64_t> rbase;
    for (int t : R) {
        from_raw = from_raw && ts[(size_t)t] % (uint64_t)HOP == 0;
        rbase.push_back(rpfx[(size_t)t] + ts[(size_t)t] / (uint64_t)HOP);
    }
    if (from_raw)
        launch_frame_rms_from_raw(d_srms, c_.up("B.rbase", rbase), d_samples, d_src, d_g, d_nt, bo.d_fpfx, NR, bo.total,
                                  FS, HOP, d_erms, st);
    else
        launch_frame_rms(d_samples, d_src, d_g, d_nt, bo.d_fpfx, NR, bo.total, FS, HOP, d_erms, st);
    uint32_t* d_eon = c_.dev<uint32_t>("B.eon", std::max<uint64_t>(bo.total, 1));
    int* d_en = c_.dev<int>("B.en", (size_t)NR);
    launch_energy_onsets(d_erms, bo.d_fpfx, d_nt, HOP, sd_powf(10.0f, -20.0f / 20.0f), d_eon, bo.d_fpfx, d_en, NR, st);
    const int kinds = hpss_on ? 3 : 2;  // spectral flux, HFC (+ HPSS)
    uint32_t* d_fon = c_.dev<uint32_t>("B.fon", kinds * std::max<uint64_t>(bo.total, 1));
    int* d_fn = c_.dev<int>("B.fn", kinds * (size_t)NR);
    float* d_fscr = c_.dev<float>("B.fscr", kinds * std::max<uint64_t>(bo.total, 1));
    const float pct = cfg_.onset_threshold_percentile;
    if (pct >= 0.0f && pct <= 1.0f)
        launch_flux_onsets(bo.SFO, bo.H, hpss_on ? d_hpe : nullptr, d_fscr, bo.d_fpfx, d_nt, HOP, pct, d_fon, bo.d_fpfx,
                           d_fn, NR, st);
    else  // detect_*_onsets return Err -> warn + empty lists (src/lib.rs:196-236)
        SDSP_HIP_CHECK(hipMemsetAsync(d_fn, 0, kinds * (size_t)NR * sizeof(int), st));
    if (hpss_on && !d_hpe)  // no frames at all: empty HPSS lists
        SDSP_HIP_CHECK(hipMemsetAsync(d_fn + 2 * NR, 0, (size_t)NR * sizeof(int), st));
    const uint64_t lists = hpss_on ? 4 : 3;
    std::vector<int> has_mags((size_t)NR);
    std::vector<uint64_t> coff((size_t)NR);
    for (int i = 0; i < NR; i++) {
        has_mags[(size_t)i] = bo.fpfx[(size_t)i + 1] > bo.fpfx[(size_t)i];
        coff[(size_t)i] = lists * bo.fpfx[(size_t)i];
    }
    int* d_hm = c_.up("B.hasm", has_mags);
    uint64_t* d_coff = c_.up("B.coff", coff);
    uint32_t* d_chosen = c_.dev<uint32_t>("B.chosen", lists * std::max<uint64_t>(bo.total, 1));
    int* d_cn = c_.dev<int>("B.cn", (size_t)NR);
    bool cons_ok = cfg_.enable_onset_consensus && cfg_.onset_consensus_tolerance_ms > 0;
    for (int k = 0; k < 4; k++) cons_ok = cons_ok && !(cfg_.onset_consensus_weights[k] < 0.0f);
    const uint32_t tol = (uint32_t)sd_f2u64((float)cfg_.onset_consensus_tolerance_ms / 1000.0f * (float)sr_);
    uint32_t* d_cscr = c_.dev<uint32_t>("B.cscr", 5 * lists * std::max<uint64_t>(bo.total, 1));
    launch_consensus(d_eon, bo.d_fpfx, d_en, d_fon, bo.d_fpfx, d_fn, bo.total, NR, tol, cons_ok, d_hm, d_chosen, d_coff,
                     d_cn, d_cscr, st, hpss_on ? 1 : 0);
    SDSP_HIP_CHECK(hipGetLastError());
    if (best.empty()) best = c_.down(bo.est, (size_t)NR);
    std::vector<int> en_h = c_.down(d_en, (size_t)NR);
    htr("B");
    tm.mark(3);
    // final tempo per track (tempogram -> legacy -> 0; legacy is never consulted on the default path,
    // see DESIGN.md "legacy estimator")
    std::vector<float> fbpm((size_t)NR, 0.0f), fconf((size_t)NR, 0.0f);
    std::vector<int> used((size_t)NR, 0);
    std::vector<int> E;  // escalated (positions in R)
    for (int i = 0; i < NR; i++) {
        TrackRes& r = res[(size_t)idx[(size_t)R[(size_t)i]]];
        const TempoEst& e = best[(size_t)i];
        r.onset_consensus = en_h[(size_t)i] > 0 ? 1.0f : 0.0f;
        if (!e.ok || !tg_on) continue;
        fbpm[(size_t)i] = e.bpm;
        fconf[(size_t)i] = e.conf;
        if (mr_on) {
            r.mr_trig = (int8_t)(e.ambiguous != 0);
            r.mr_used = 0;
            r.perc_trig = (int8_t)(e.ambiguous && e.trap_low);
            if (e.ambiguous) E.push_back(i);
        }
    }
    if (dbg_on && mr_on) {  // src/lib.rs:461-487: the base estimate and its candidate list
        const std::vector<TempoEst> be = best.empty() ? c_.down(bo.est, (size_t)NR) : best;
        const std::vector<float> bc = c_.down(bo.cand, (size_t)NR * (size_t)bin.cand_cap * 4);
        for (int i = 0; i < NR; i++) {
            if (!be[(size_t)i].ok) continue;
            TrackDbg& t = tdbg[(size_t)i];
            t.base = true;
            t.est = be[(size_t)i];
            for (int c = 0; c < std::min(be[(size_t)i].n_cands, bin.cand_cap); c++) {
                const float* q = bc.data() + ((size_t)i * (size_t)bin.cand_cap + (size_t)c) * 4;
                t.base_c.push_back({q[0], q[1], q[2], q[3]});
            }
        }
    }
    float* d_fbpm = c_.up("B.fbpm", fbpm);
    float* d_fconf = c_.up("B.fconf", fconf);
    int* d_used = c_.up("B.used", used);
    // ---------------- C: escalation (multi_resolution.rs:205-901) ----------------
    TempoEst* d_mr_all = nullptr;  // multi-res estimates of the escalated tracks (E order)
    // hop_size != 512: the escalation's own hop-512 candidate lists (E order; emitted for the
    // tracks that take the multi-res estimate, src/lib.rs:546,686) and the E position of each track
    std::vector<float> c512_h;
    std::vector<int> n512_own, epos((size_t)NR, -1);
    int c512_cap = 0;
    if (mr_on && !E.empty()) {
        const int NE = (int)E.size();
        const int top_k = (int)std::max<uint64_t>(cfg_.tempogram_multi_res_top_k, 1);
        const int aux_k = std::min(std::max(top_k * 4, 25), 200);
        TempoPassIn ein;
        ein.samples = d_samples;
        for (int i : E) {
            ein.src_off.push_back(bin.src_off[(size_t)i]);
            ein.gain_h.push_back(bin.gain_h[(size_t)i]);
            ein.n_trim.push_back(bin.n_trim[(size_t)i]);
        }
        ein.want_onsets = false;
        ein.gate = 0;
        // multi_resolution.rs:237-239 recomputes the STFT at hops 256, 512 and 1024 of the trimmed
        // samples.  At hop_size 512 the base pass is the hop-512 one; otherwise the escalated
        // tracks get their own hop-512 pass (top_k candidates, :273) first.  The hop-256 and
        // hop-1024 passes read the hop-512 rows they share with it (SDSP_NO_ROW_REUSE: control).
        const bool own512 = HOP != 512;
        TempoPassOut o256, o512, o1024;
        if (own512) {
            ein.hop = 512;
            ein.top_n = top_k;
            ein.cand_cap = top_k;
            ein.mr_nov = true;
            tempo_pass("C512.", ein, o512);
            ein.mr_nov = false;
        }
        const TempoPassOut& b512 = own512 ? o512 : bo;
        ein.base_mags = b512.mags;
        ein.base_fmax = b512.fmax;
        for (int k = 0; k < NE; k++) ein.base_row0.push_back(b512.fpfx[own512 ? (size_t)k : (size_t)E[(size_t)k]]);
        ein.top_n = aux_k;
        ein.cand_cap = aux_k;
        const bool reuse_on = test_hooks().no_row_reuse.load() == 0;  // the tests' control (sdsp_debug_set_schedule)
        ein.hop = 256;
        ein.reuse = reuse_on ? 2 : 0;
        tempo_pass("C256.", ein, o256);
        ein.hop = 1024;
        ein.reuse = reuse_on ? 1 : 0;
        tempo_pass("C1024.", ein, o1024);
        std::vector<TempoPassOut*> mr_passes = {&o256, &o1024};
        if (own512) mr_passes.push_back(&o512);
        for (TempoPassOut* o : mr_passes) {
            times_.stft2048_ms += o->stft_ms;
            times_.stft2048_launches += o->stft_launch;
            times_.stft2048_frames += o->stft_frames;
            times_.stft2048_bytes += o->stft_bytes;
            times_.features_ms += o->feat_ms;
            times_.tempogram_ms += o->tempo_ms;
        }
        std::vector<TempoEst> e256 = c_.down(o256.est, (size_t)NE), e1024 = c_.down(o1024.est, (size_t)NE);
        std::vector<int> n256((size_t)NE), n1024((size_t)NE), n512((size_t)NR);
        for (int k = 0; k < NE; k++) {
            n256[(size_t)k] = e256[(size_t)k].ok ? e256[(size_t)k].n_cands : -1;
            n1024[(size_t)k] = e1024[(size_t)k].ok ? e1024[(size_t)k].n_cands : -1;
        }
        if (own512) {  // E order; -1: the hop-512 tempogram failed (multi_resolution returns Err)
            const std::vector<TempoEst> e512 = c_.down(o512.est, (size_t)NE);
            n512.assign((size_t)NE, 0);
            for (int k = 0; k < NE; k++)
                n512[(size_t)k] = e512[(size_t)k].ok ? std::min(e512[(size_t)k].n_cands, top_k) : -1;
            if (cfg_.emit_tempogram_candidates) {
                c512_h = c_.down(o512.cand, (size_t)NE * (size_t)top_k * 4);
                n512_own = n512;
                c512_cap = top_k;
                for (int k = 0; k < NE; k++) epos[(size_t)E[(size_t)k]] = k;
            }
        } else {
            for (int i = 0; i < NR; i++) n512[(size_t)i] = std::min(best[(size_t)i].n_cands, top_k);
        }
        int* d_n256 = c_.up("C.n256", n256);
        int* d_n1024 = c_.up("C.n1024", n1024);
        int* d_n512 = c_.up("C.n512", n512);
        int* d_E = c_.up("C.E", E);
        MrParams mp{};
        mp.min_bpm = cfg_.min_bpm;
        mp.max_bpm = cfg_.max_bpm;
        mp.tol = sd_maxf(2.0f, cfg_.bpm_resolution);
        mp.w512 = cfg_.tempogram_multi_res_w512;
        mp.w256 = cfg_.tempogram_multi_res_w256;
        mp.w1024 = cfg_.tempogram_multi_res_w1024;
        mp.dt = cfg_.tempogram_multi_res_double_time_512_factor;
        mp.margin_thr = cfg_.tempogram_multi_res_margin_threshold;
        mp.human_prior = cfg_.tempogram_multi_res_use_human_prior;
        mp.top_k = top_k;
        mp.band = 1;  // src/lib.rs:509 always passes Some(band_cfg)
        mp.sr = (int)sr_;
        mp.hop512 = 512;
        mp.own512 = own512 ? 1 : 0;
        TempoEst* d_mr = c_.dev<TempoEst>("C.mr", (size_t)NE);
        d_mr_all = d_mr;
        MrDbg* d_mdbg = dbg_on ? c_.dev<MrDbg>("C.mrdbg", (size_t)NE) : nullptr;
        launch_multires(d_E, NE, o256.cand, d_n256, b512.cand, d_n512, o1024.cand, d_n1024, ein.cand_cap,
                        own512 ? top_k : bin.cand_cap, ein.cand_cap, bo.est, b512.nov_mr, b512.d_fpfx, mp, d_mr, d_used,
                        d_fbpm, d_fconf, st, d_mdbg);
        SDSP_HIP_CHECK(hipGetLastError());
        if (dbg_on) {  // multi_resolution.rs:304-403, 707-860 and src/lib.rs:547-573
            const int cap512 = own512 ? top_k : bin.cand_cap;
            const std::vector<float> h256 = c_.down(o256.cand, (size_t)NE * (size_t)ein.cand_cap * 4);
            const std::vector<float> h1024 = c_.down(o1024.cand, (size_t)NE * (size_t)ein.cand_cap * 4);
            const std::vector<float> h512 =
                c_.down(b512.cand, (size_t)(own512 ? NE : NR) * (size_t)cap512 * 4);
            const std::vector<TempoEst> hmr = c_.down(d_mr, (size_t)NE);
            const std::vector<MrDbg> hmd = c_.down(d_mdbg, (size_t)NE);
            auto list = [](const std::vector<float>& h, size_t row, int cap, int n) {
                std::vector<Cand4> v;
                for (int c = 0; c < n; c++) {
                    const float* q = h.data() + (row * (size_t)cap + (size_t)c) * 4;
                    v.push_back({q[0], q[1], q[2], q[3]});
                }
                return v;
            };
            for (int k = 0; k < NE; k++) {
                const int i = E[(size_t)k];
                TrackDbg& t = tdbg[(size_t)i];
                const int j512 = own512 ? k : i;
                if (!hmr[(size_t)k].ok || n256[(size_t)k] < 0 || n1024[(size_t)k] < 0 || n512[(size_t)j512] < 0) continue;
                t.mr = true;
                t.c256 = list(h256, (size_t)k, ein.cand_cap, n256[(size_t)k]);
                t.c512 = list(h512, (size_t)j512, cap512, n512[(size_t)j512]);
                t.c1024 = list(h1024, (size_t)k, ein.cand_cap, n1024[(size_t)k]);
                t.mr_est = hmr[(size_t)k];
                t.md = hmd[(size_t)k];
            }
        }
        used = c_.down(d_used, (size_t)NR);
        for (int i : E) {
            if (used[(size_t)i]) res[(size_t)idx[(size_t)R[(size_t)i]]].mr_used = 1;
        }
        if (cfg_.emit_tempogram_candidates) {
            // the multi-res candidate list is hop 512's (top_k), re-flagged against the fused BPM
            std::vector<TempoEst> mr = c_.down(d_mr, (size_t)NE);
            std::vector<float> fb = c_.down(d_fbpm, (size_t)NR);
            (void)mr;
            fbpm = fb;
        }
    }
    std::vector<float> fbpm_h = c_.down(d_fbpm, (size_t)NR), fconf_h = c_.down(d_fconf, (size_t)NR);
    htr("C");
    // ---------------- C': percussive tempogram fallback (src/lib.rs:582-683) ----------------
    std::vector<std::vector<float>> perc_cands((size_t)NR);  // emitted candidates of tracks that took it
    std::vector<uint8_t> perc_took((size_t)NR, 0);
    if (perc_on) {
        std::vector<int> Q;  // positions in R
        for (int i = 0; i < NR; i++) {
            const TempoEst& e = best[(size_t)i];
            if (!e.ok) continue;
            res[(size_t)idx[(size_t)R[(size_t)i]]].perc_used = 0;
            if (e.ambiguous && e.trap_low) Q.push_back(i);
        }
        const int NQ = (int)Q.size();
        if (NQ > 0 && d_P0) {
            TempoPassIn pin;
            pin.hop = HOP;
            pin.samples = d_samples;
            std::vector<uint64_t> qpfx(1, 0);
            for (int i : Q) {
                pin.src_off.push_back(bin.src_off[(size_t)i]);
                pin.gain_h.push_back(bin.gain_h[(size_t)i]);
                pin.n_trim.push_back(bin.n_trim[(size_t)i]);
                qpfx.push_back(qpfx.back() + (bo.fpfx[(size_t)i + 1] - bo.fpfx[(size_t)i]));
            }
            pin.want_onsets = false;
            pin.top_n = bin.top_n;
            pin.cand_cap = bin.cand_cap;
            pin.gate = 0;
            if (hpss_on) {  // S holds every track: gather Q's rows (S == Q otherwise)
                float* pq = c_.dev<float>("P.in", std::max<uint64_t>(qpfx.back(), 1) * s2_);
                float* pm = c_.dev<float>("P.inmax", std::max<uint64_t>(qpfx.back(), 1));
                for (int k = 0; k < NQ; k++) {
                    const uint64_t F = qpfx[(size_t)k + 1] - qpfx[(size_t)k], r0 = bo.fpfx[(size_t)Q[(size_t)k]];
                    if (F == 0) continue;
                    SDSP_HIP_CHECK(hipMemcpyAsync(pq + qpfx[(size_t)k] * s2_, d_P0 + r0 * s2_,
                                                  F * s2_ * sizeof(float), hipMemcpyDeviceToDevice, st));
                    SDSP_HIP_CHECK(hipMemcpyAsync(pm + qpfx[(size_t)k], d_hfmax + r0, F * sizeof(float),
                                                  hipMemcpyDeviceToDevice, st));
                }
                pin.mags_in = pq;
                pin.fmax_in = pm;
            } else {
                pin.mags_in = d_P0;
                pin.fmax_in = d_hfmax;
            }
            TempoPassOut po;
            tempo_pass("P.", pin, po);
            times_.features_ms += po.feat_ms;
            times_.tempogram_ms += po.tempo_ms;
            std::vector<TempoEst> pe = c_.down(po.est, (size_t)NQ);
            std::vector<TempoEst> mr_h;
            if (d_mr_all) mr_h = c_.down(d_mr_all, E.size());
            std::vector<int> epos((size_t)NR, -1);
            for (size_t k = 0; k < E.size(); k++) epos[(size_t)E[k]] = (int)k;
            std::vector<float> pc_h;
            if (cfg_.emit_tempogram_candidates) pc_h = c_.down(po.cand, (size_t)NQ * (size_t)pin.cand_cap * 4);
            bool changed = false;
            for (int k = 0; k < NQ; k++) {
                const int i = Q[(size_t)k];
                const TempoEst& p = pe[(size_t)k];
                if (!p.ok) continue;  // "Percussive tempogram fallback failed" -> not used
                const TempoEst& b = best[(size_t)i];
                const float cb = fbpm_h[(size_t)i], cc = fconf_h[(size_t)i];
                const int ca = (used[(size_t)i] && epos[(size_t)i] >= 0) ? mr_h[(size_t)epos[(size_t)i]].agree : b.agree;
                const float rel = cb > 1e-6f ? sd_maxf(p.bpm / cb, cb / p.bpm) : 1.0f;
                const bool fam = sd_absf(rel - 2.0f) < 0.05f || sd_absf(rel - 1.5f) < 0.05f ||
                                 sd_absf(rel - (4.0f / 3.0f)) < 0.05f || sd_absf(rel - (3.0f / 2.0f)) < 0.05f ||
                                 sd_absf(rel - (2.0f / 3.0f)) < 0.05f || sd_absf(rel - (3.0f / 4.0f)) < 0.05f;
                const bool forbid = cb <= 180.0f && p.bpm > 180.0f;
                const bool base_low_trap = b.trap_low || b.bpm < 95.0f;
                const bool in_common = p.bpm >= 70.0f && p.bpm <= 180.0f;
                const bool better = !forbid && fam && in_common &&
                                    (p.conf >= cc + 0.04f || (base_low_trap && p.conf >= cc * 0.85f) ||
                                     (p.agree > ca && p.conf >= cc * 0.92f));
                if (!better) continue;
                fbpm_h[(size_t)i] = p.bpm;
                fconf_h[(size_t)i] = p.conf;
                res[(size_t)idx[(size_t)R[(size_t)i]]].perc_used = 1;
                perc_took[(size_t)i] = 1;
                changed = true;
                if (cfg_.emit_tempogram_candidates)
                    perc_cands[(size_t)i].assign(pc_h.begin() + (long)((size_t)k * (size_t)pin.cand_cap * 4),
                                                 pc_h.begin() + (long)((size_t)k * (size_t)pin.cand_cap * 4 +
                                                                       (size_t)p.n_cands * 4));
            }
            if (changed) {
                SDSP_HIP_CHECK(hipMemcpyAsync(d_fbpm, c_.keep_bytes(fbpm_h), (size_t)NR * sizeof(float),
                                              hipMemcpyHostToDevice, st));
                SDSP_HIP_CHECK(hipMemcpyAsync(d_fconf, c_.keep_bytes(fconf_h), (size_t)NR * sizeof(float),
                                              hipMemcpyHostToDevice, st));
            }
        }
        htr("C perc");
    }
    // ---------------- C'': legacy estimator (src/lib.rs:294-329) and the BPM choice (:814-900) ------
    if (cfg_.force_legacy_bpm || cfg_.enable_bpm_fusion)
        legacy_select(bin, d_chosen, d_coff, d_cn, R, idx, res, fbpm_h, fconf_h, d_fbpm, d_fconf);
    tm.mark(4);
    if (bpm_only_) {
        for (int i = 0; i < NR; i++) {
            TrackRes& r = res[(size_t)idx[(size_t)R[(size_t)i]]];
            if (r.status != SDSP_OK) continue;
            r.bpm = fbpm_h[(size_t)i];
            r.bpm_conf = fconf_h[(size_t)i];
        }
        htr("results (bpm only)");
        return;
    }
    // ---------------- D: beat grid ----------------
    std::vector<int> ident((size_t)NR);
    std::vector<uint64_t> boff((size_t)NR + 1, 0);
    std::vector<int> bcap((size_t)NR);
    for (int i = 0; i < NR; i++) {
        ident[(size_t)i] = i;
        const uint64_t n = bin.n_trim[(size_t)i];
        const uint64_t dur_s = n / std::max<uint32_t>(sr_, 1) + 1;
        const uint64_t F = bo.fpfx[(size_t)i + 1] - bo.fpfx[(size_t)i];
        const uint64_t cap = std::max<uint64_t>(12 * dur_s + 64, 3 * F + 8);
        bcap[(size_t)i] = (int)cap;
        boff[(size_t)i + 1] = boff[(size_t)i] + cap;
    }
    int* d_ident = c_.up("D.ident", ident);
    uint64_t* d_boff = c_.up("D.boff", boff);
    int* d_bcap = c_.up("D.bcap", bcap);
    float* d_bscr = c_.dev<float>("D.bscr", 4 * boff[(size_t)NR]);
    float* d_beats = c_.dev<float>("D.beats", boff[(size_t)NR]);
    float* d_downs = c_.dev<float>("D.downs", boff[(size_t)NR]);
    BeatOut* d_bout = c_.dev<BeatOut>("D.bout", (size_t)NR);
    launch_beat(d_ident, NR, d_chosen, d_coff, d_cn, sr_, d_fbpm, d_fconf, d_bscr, d_boff, d_bcap, d_beats, d_downs,
                d_bout, st);
    SDSP_HIP_CHECK(hipGetLastError());
    tm.mark(5);
    tm.mark(6);
    const bool beat_sync = cfg_.enable_key_beat_synchronous && !cfg_.enable_key_log_frequency;
    // the previous sub-batch's key results (its key work ran ahead of this one's on the key stream),
    // and the exact rerun of its near-decision tracks on the main stream
    rerun_near(d_samples, in_off, n_raw, finish_key(res), res);
    // late join by default (+2 % in alternating bench runs on one box, 2,350 vs 2,301 tracks/s:
    // the main stream otherwise idles ~45 ms per sub-batch waiting for the key tail);
    // no_key_defer (sdsp_debug_set_schedule) joins at the end of each sub-batch (the tests' control)
    const bool defer_key =
        NK > 0 && !beat_sync && !serial_streams && !dbg_on && test_hooks().no_key_defer.load() == 0;
    if (defer_key) {
        key_pending_.reset(new KeyPending());
        key_pending_->kt = std::move(ktp);
        key_pending_->d_kout = d_kout;
        for (int k = 0; k < NK; k++) key_pending_->at.push_back((size_t)idx[(size_t)R[(size_t)K[(size_t)k]]]);
        ktail.kp = kp;
        key_pending_->tail = std::move(ktail);
    } else if (NK > 0) {  // join the key stream
        SDSP_HIP_CHECK(hipStreamWaitEvent(st, kt.ev[2], 0));
        kout = c_.down(d_kout, (size_t)NK);
        htr("E join");
        times_.stft8192_ms += kt.ms(0, 1);
        times_.key_ms += kt.ms(1, 2);
    }
    // ---------------- results ----------------
    uint64_t* d_bpfx = c_.dev<uint64_t>("D.bpfx", 2 * ((size_t)NR + 1));
    float* d_cbeats = c_.dev<float>("D.cbeats", boff[(size_t)NR]);
    float* d_cdowns = c_.dev<float>("D.cdowns", boff[(size_t)NR]);
    launch_beat_compact(NR, d_bout, d_boff, d_beats, d_downs, d_bpfx, d_cbeats, d_cdowns, st);
    SDSP_HIP_CHECK(hipGetLastError());
    std::vector<BeatOut> bout = c_.down(d_bout, (size_t)NR);
    std::vector<uint64_t> bpfx = c_.down(d_bpfx, 2 * ((size_t)NR + 1));
    std::vector<float> beats_h = c_.down(d_cbeats, bpfx[(size_t)NR]);
    std::vector<float> downs_h = c_.down(d_cdowns, bpfx[2 * (size_t)NR + 1]);
    std::vector<float> cand_h;
    if (cfg_.emit_tempogram_candidates) cand_h = c_.down(bo.cand, (size_t)NR * (size_t)bin.cand_cap * 4);
    htr("D down");
    // beat-synchronous chroma (src/lib.rs:1121-1133): for key tracks with a non-empty beat grid the
    // chroma rows are the beat intervals' mean frame chroma; the key vote is re-run on them
    if (beat_sync && NK > 0) {
        std::vector<int> sel, sel_id;
        std::vector<uint64_t> sb_off, rpfx(1, 0), sseg(1, 0);
        for (int k = 0; k < NK; k++) {
            const int i = K[(size_t)k];
            const int nb = bout[(size_t)i].ok > 0 ? bout[(size_t)i].n_beats : 0;
            if (nb < 1) continue;
            sel.push_back(k);
            sel_id.push_back((int)sel_id.size());
            sb_off.push_back(bpfx[(size_t)i]);
            const uint64_t rows = (uint64_t)nb - 1;
            rpfx.push_back(rpfx.back() + rows);
            sseg.push_back(sseg.back() + (uint64_t)KV_ROW * seg_rows(rows));
        }
        const int NS = (int)sel.size();
        if (NS > 0) {
            const uint64_t total8 = kpfx.back();
            ChromaParams cp = chroma_params(cfg_, sr_, 0, B8, fres8, ks_);
            cp.gate_small = 0;  // extract_beat_synchronous_chroma takes the offset as is
            float* fc = c_.dev<float>("E.bs_fc", total8 * 12);
            float* fe = c_.dev<float>("E.bs_fe", total8);
            launch_chroma(0, mags8, d_kpfx, d_ktile, d_kid, NK, ktile.back(), cp, d_tune, fc, fe, st);
            int* d_sel = c_.up("E.bs_sel", sel);
            int* d_sid = c_.up("E.bs_id", sel_id);
            uint64_t* d_sboff = c_.up("E.bs_boff", sb_off);
            uint64_t* d_rpfx = c_.up("E.bs_rpfx", rpfx);
            uint64_t* d_sseg = c_.up("E.bs_seg", sseg);
            const uint64_t rows = std::max<uint64_t>(rpfx.back(), 1);
            float* bc = c_.dev<float>("E.bs_chroma", rows * 12);
            float* be = c_.dev<float>("E.bs_energy", rows);
            const float fd = (float)KHOP / (float)sr_;
            launch_beat_sync(d_sel, NS, d_kpfx, fc, fe, d_cbeats, d_sboff, d_rpfx, fd, bc, be, st);
            float* bcs = c_.dev<float>("E.bs_chroma_s", rows * 12);
            float* bw = c_.dev<float>("E.bs_weights", rows);
            float* bscr = c_.dev<float>("E.bs_segscr", std::max<uint64_t>(sseg.back(), 1));
            KeyOut* d_bko = c_.dev<KeyOut>("E.bs_kout", (size_t)NS);
            launch_key_vote(d_sid, NS, d_rpfx, bc, be, bcs, bw, bscr, d_sseg, d_tpl, kp, d_bko, st);
            SDSP_HIP_CHECK(hipGetLastError());
            std::vector<KeyOut> bko = c_.down(d_bko, (size_t)NS);
            for (int j = 0; j < NS; j++) kout[(size_t)sel[(size_t)j]] = bko[(size_t)j];
        }
        htr("E beat-sync");
    }
    times_.beat_ms += tm.ms(4, 5);
    for (int i = 0; i < NR; i++) {
        TrackRes& r = res[(size_t)idx[(size_t)R[(size_t)i]]];
        if (r.status != SDSP_OK) continue;  // a legacy-estimator error propagated
        r.bpm = fbpm_h[(size_t)i];
        r.bpm_conf = fconf_h[(size_t)i];
        const BeatOut& b = bout[(size_t)i];
        if (b.ok < 0) {
            r.status = SDSP_ERR_PROCESSING;
            r.err = "Processing error: beat buffer capacity exceeded";
            continue;
        }
        if (b.ok > 0) {
            const uint64_t ob = bpfx[(size_t)i], od = bpfx[(size_t)NR + 1 + (size_t)i];
            r.beats.assign(beats_h.begin() + (long)ob, beats_h.begin() + (long)(ob + b.n_beats));
            r.downs.assign(downs_h.begin() + (long)od, downs_h.begin() + (long)(od + b.n_down));
            r.stability = b.stability;
        }
        if (cfg_.emit_tempogram_candidates && perc_took[(size_t)i]) {  // chosen_cands = p_cands (:661-664)
            r.has_cands = true;
            const std::vector<float>& pc = perc_cands[(size_t)i];
            for (size_t k = 0; k + 4 <= pc.size(); k += 4) {
                sdsp_tempo_candidate tc{pc[k], pc[k + 1], pc[k + 2], pc[k + 3], (uint8_t)(sd_absf(pc[k] - r.bpm) < 0.75f)};
                r.cands.push_back(tc);
            }
        } else if (cfg_.emit_tempogram_candidates && r.mr_used == 1 && epos[(size_t)i] >= 0) {
            r.has_cands = true;  // the escalation's own hop-512 list (hop_size != 512)
            const int k = epos[(size_t)i];
            for (int c = 0; c < n512_own[(size_t)k]; c++) {
                const float* cc = c512_h.data() + ((size_t)k * (size_t)c512_cap + (size_t)c) * 4;
                sdsp_tempo_candidate tc{cc[0], cc[1], cc[2], cc[3], (uint8_t)(sd_absf(cc[0] - r.bpm) < 0.75f)};
                r.cands.push_back(tc);
            }
        } else if (cfg_.emit_tempogram_candidates && best[(size_t)i].ok && tg_on) {
            r.has_cands = true;
            int n = best[(size_t)i].n_cands;
            if (mr_on && r.mr_used == 1) n = std::min(n, (int)std::max<uint64_t>(cfg_.tempogram_multi_res_top_k, 1));
            for (int k = 0; k < n; k++) {
                const float* cc = cand_h.data() + ((size_t)i * (size_t)bin.cand_cap + (size_t)k) * 4;
                sdsp_tempo_candidate tc{cc[0], cc[1], cc[2], cc[3], (uint8_t)(sd_absf(cc[0] - r.bpm) < 0.75f)};
                r.cands.push_back(tc);
            }
        }
    }
    for (int k = 0; k < NK && !defer_key; k++) {
        TrackRes& r = res[(size_t)idx[(size_t)R[(size_t)K[(size_t)k]]]];
        const KeyOut& ko = kout[(size_t)k];
        if (!ko.ok) continue;
        r.key_mode = ko.mode;
        r.key_tonic = ko.tonic;
        r.key_conf = ko.conf;
        r.key_clarity = ko.clarity;
        r.key_near = ko.near;
    }
    if (dbg_on) {
        if (NK > 0) {  // src/lib.rs:1471-1538 (the beat-synchronous re-vote keeps the frame-level record)
            const std::vector<KeyDbg> kd = c_.down(d_kdbg, (size_t)NK);
            const std::vector<float> tu = d_tune ? c_.down(d_tune, (size_t)NK) : std::vector<float>((size_t)NK, 0.0f);
            for (int k = 0; k < NK; k++) {
                const KeyOut& ko = kout[(size_t)k];
                if (!ko.ok) continue;
                TrackDbg& t = tdbg[(size_t)K[(size_t)k]];
                t.key = true;
                t.ko = ko;
                t.kd = kd[(size_t)k];
                t.tuning = tu[(size_t)k];
            }
        }
        for (int i = 0; i < NR; i++) print_debug(cfg_, tdbg[(size_t)i]);
    }
    htr("results");
}

namespace {

char* dup_str(const std::string& s) {
    char* p = (char*)std::malloc(s.size() + 1);
    std::memcpy(p, s.c_str(), s.size() + 1);
    return p;
}
float* dup_f(const std::vector<float>& v) {
    if (v.empty()) return nullptr;
    float* p = (float*)std::malloc(v.size() * sizeof(float));
    std::memcpy(p, v.data(), v.size() * sizeof(float));
    return p;
}

// result assembly + warnings (src/lib.rs:1561-1619)
void fill_result(const TrackRes& r, uint32_t sr, float ms, sdsp_result* o) {
    std::memset(o, 0, sizeof(*o));
    o->status = r.status;
    o->tempogram_multi_res_triggered = o->tempogram_multi_res_used = -1;
    o->tempogram_percussive_triggered = o->tempogram_percussive_used = -1;
    if (r.status != SDSP_OK) {
        std::snprintf(o->error_message, sizeof o->error_message, "%s", r.err.c_str());
        return;
    }
    o->bpm = r.bpm;
    o->bpm_confidence = r.bpm_conf;
    o->key_mode = r.key_mode;
    o->key_tonic = (uint32_t)r.key_tonic;
    o->key_confidence = r.key_conf;
    o->key_clarity = r.key_clarity;
    o->beats = dup_f(r.beats);
    o->n_beats = r.beats.size();
    o->downbeats = dup_f(r.downs);
    o->n_downbeats = r.downs.size();
    o->bars = dup_f(r.downs);
    o->n_bars = r.downs.size();
    o->grid_stability = r.stability;
    o->duration_seconds = r.duration;
    o->sample_rate = sr;
    o->processing_time_ms = ms;
    std::snprintf(o->algorithm_version, sizeof o->algorithm_version, "0.1.0-alpha");
    o->onset_method_consensus = r.onset_consensus;
    o->methods_used = 7;
    std::vector<std::string> w;
    if (r.bpm == 0.0f) w.push_back("BPM detection failed: insufficient onsets or estimation error");
    if (r.stability < 0.5f) w.push_back("Low beat grid stability: " + fmt2(r.stability) + " (may indicate tempo variation)");
    if (r.key_conf < 0.3f)
        w.push_back("Low key detection confidence: " + fmt2(r.key_conf) + " (may indicate ambiguous or atonal music)");
    if (r.key_clarity < 0.2f) {
        w.push_back("Low key clarity: " + fmt2(r.key_clarity) + " (track may be atonal or have weak tonality)");
        o->flags |= SDSP_FLAG_WEAK_TONALITY;
    }
    o->n_warnings = w.size();
    if (!w.empty()) {
        o->warnings = (char**)std::malloc(w.size() * sizeof(char*));
        for (size_t i = 0; i < w.size(); i++) o->warnings[i] = dup_str(w[i]);
    }
    o->has_tempogram_candidates = r.has_cands;
    if (r.has_cands && !r.cands.empty()) {
        o->n_tempogram_candidates = r.cands.size();
        o->tempogram_candidates = (sdsp_tempo_candidate*)std::malloc(r.cands.size() * sizeof(sdsp_tempo_candidate));
        std::memcpy(o->tempogram_candidates, r.cands.data(), r.cands.size() * sizeof(sdsp_tempo_candidate));
    }
    o->tempogram_multi_res_triggered = r.mr_trig;
    o->tempogram_multi_res_used = r.mr_used;
    o->tempogram_percussive_triggered = r.perc_trig;
    o->tempogram_percussive_used = r.perc_used;
}

// One device-resident batch on `device`.  The engine's main stream first waits for `user_stream`
// (everything queued on it so far) and for `wait_ev` (a copy's completion), whichever are given.
// The batch on a context whose mutex the caller holds (run_device, and sdsp_analyze_audio's
// direct path, which stages its one track into a context buffer under the same lock).
int32_t run_locked(DeviceCtx& d, const float* d_samples, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                   uint32_t sr, const sdsp_config* cfg, void* user_stream, sdsp_result* outs, int stages,
                   hipEvent_t wait_ev) {
    if (stages != SDSP_STAGES_FULL && stages != SDSP_STAGES_BPM_ONLY) throw HipError("unknown stage mask");
    if (user_stream) {
        hipEvent_t ev;
        SDSP_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        SDSP_HIP_CHECK(hipEventRecord(ev, (hipStream_t)user_stream));
        SDSP_HIP_CHECK(hipStreamWaitEvent(d.stream, ev, 0));
        SDSP_HIP_CHECK(hipEventDestroy(ev));
    }
    if (wait_ev) SDSP_HIP_CHECK(hipStreamWaitEvent(d.stream, wait_ev, 0));
    auto t0 = std::chrono::steady_clock::now();
    std::vector<uint64_t> off(offsets, offsets + n), ln(lens, lens + n);
    std::vector<TrackRes> res;
    Pipeline p(d, *cfg, sr, stages);
    try {
        p.run(d_samples, off, ln, res);
        // Certified block energies: a track whose key vote had an energy-dependent
        // decision within its margin (KeyOut::near) has its key path run again with the reference's
        // sequential frame-energy fold, and those key fields replace its own (everything else is
        // independent of the key energies).
        std::vector<size_t> near;
        d.last_near.assign(res.size(), 0);
        for (size_t i = 0; i < res.size(); i++) {
            if (res[i].key_near) d.last_near[i] = (uint8_t)res[i].key_near;
            if (res[i].key_near && !res[i].key_rerun) near.push_back(i);  // the last sub-batch's
        }
        if (!near.empty()) {
            const sdsp_stage_times first = d.last;
            std::vector<uint64_t> o2, l2;
            for (size_t i : near) o2.push_back(off[i]), l2.push_back(ln[i]);
            std::vector<TrackRes> r2;
            Pipeline px(d, *cfg, sr, stages, true, true);
            px.run(d_samples, o2, l2, r2);
            for (size_t j = 0; j < near.size(); j++) {
                TrackRes& r = res[near[j]];
                if (r2[j].status != SDSP_OK) {  // (the same front end as the main pass) uncertified: fail
                    r.status = SDSP_ERR_PROCESSING;
                    r.err = "Processing error: key certification rerun failed (" + r2[j].err + ")";
                    continue;
                }
                r.key_mode = r2[j].key_mode;
                r.key_tonic = r2[j].key_tonic;
                r.key_conf = r2[j].key_conf;
                r.key_clarity = r2[j].key_clarity;
            }
            // the call's stage times stay the main pass's; the rerun is reported beside them
            const double rerun_ms = d.last.total_ms;
            d.last = first;
            d.last.key_reruns += near.size();
            d.last.rerun_ms += rerun_ms;
            d.last.total_ms += rerun_ms;
        }
    } catch (...) {
        // a sub-batch may have queued key-stream work (the late join) before a later one threw:
        // nothing of this call may still run on the engine's streams once the context lock is
        // released, or the next call's uploads into the same context buffers would race it
        for (hipStream_t s : d.own) (void)hipStreamSynchronize(s);
        throw;
    }
    const float ms = (float)(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() /
                             (double)std::max<uint64_t>(n, 1));
    for (uint64_t i = 0; i < n; i++) fill_result(res[(size_t)i], sr, ms, &outs[i]);
    return SDSP_OK;
}

int32_t run_device(int device, const float* d_samples, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                   uint32_t sr, const sdsp_config* cfg, void* user_stream, sdsp_result* outs,
                   int stages = SDSP_STAGES_FULL, hipEvent_t wait_ev = nullptr) {
    DeviceCtx& d = device_ctx(device);
    std::lock_guard<std::mutex> lk(d.mu);
    SDSP_HIP_CHECK(hipSetDevice(device));
    return run_locked(d, d_samples, offsets, lens, n, sr, cfg, user_stream, outs, stages, wait_ev);
}

}  // namespace
}  // namespace sdsp

using namespace sdsp;

namespace sdsp {
namespace {
struct Slot {
    float* d = nullptr;
    uint64_t cap = 0;  // floats
    hipEvent_t ready = nullptr;
};
// A device's staging area: its copy stream and two HBM slots.  Areas are pooled per device and
// reused by later calls (grow-only slots, like the engine's own buffers), so a repeated call
// creates no stream, event or allocation; concurrent callers on one device take separate areas.
struct DeviceStage {
    int dev = 0;
    hipStream_t copy = nullptr;
    Slot slot[2];
};
std::mutex g_stage_mu;
std::map<int, std::vector<DeviceStage*>>* g_stage_free = new std::map<int, std::vector<DeviceStage*>>();  // never freed:
// the areas outlive the call and are released with the process (no HIP calls at static teardown)
DeviceStage* stage_acquire(int dev) {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    auto& v = (*g_stage_free)[dev];
    if (!v.empty()) {
        DeviceStage* ds = v.back();
        v.pop_back();
        return ds;
    }
    DeviceStage* ds = new DeviceStage();
    ds->dev = dev;
    return ds;
}
void stage_release(DeviceStage* ds) {
    if (ds->copy) {  // nothing may still be copying into the slots the next caller receives
        (void)hipSetDevice(ds->dev);
        (void)hipStreamSynchronize(ds->copy);
    }
    std::lock_guard<std::mutex> lk(g_stage_mu);
    (*g_stage_free)[ds->dev].push_back(ds);
}
// test hook (sdsp_debug_set_test_hooks): the worker devices of sdsp_analyze_batch, repeats
// allowed (two workers on device 0 exercise the multi-device chunk path on a one-GPU box)
// (compiled only into the test build, -DSDSP_TEST_HOOKS: the shipping library cannot be re-routed)
std::vector<int> device_list_override(int ndev) {
    std::vector<int> devs;
#ifdef SDSP_TEST_HOOKS
    for (int v : test_hooks_devices())
        if (v >= 0 && v < ndev) devs.push_back(v);
#endif
    return devs;
}
}  // namespace
}  // namespace sdsp


extern "C" {

int32_t sdsp_analyze_batch_device(const float* d_samples, const uint64_t* offsets, const uint64_t* lens,
                                  uint64_t n_tracks, uint32_t sample_rate, const sdsp_config* cfg, int32_t device,
                                  void* stream, sdsp_result* outs) {
    return sdsp_analyze_batch_device_ex(d_samples, offsets, lens, n_tracks, sample_rate, cfg, device, stream,
                                        SDSP_STAGES_FULL, outs);
}

int32_t sdsp_analyze_batch_device_ex(const float* d_samples, const uint64_t* offsets, const uint64_t* lens,
                                     uint64_t n_tracks, uint32_t sample_rate, const sdsp_config* cfg, int32_t device,
                                     void* stream, int32_t stages, sdsp_result* outs) {
    try {
        return run_device(device, d_samples, offsets, lens, n_tracks, sample_rate, cfg, stream, outs, stages);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "sdsp_analyze_batch_device: %s\n", e.what());
        for (uint64_t i = 0; i < n_tracks; i++) {
            std::memset(&outs[i], 0, sizeof(outs[i]));
            outs[i].status = SDSP_ERR_PROCESSING;
            std::snprintf(outs[i].error_message, sizeof outs[i].error_message, "Processing error: %s", e.what());
        }
        return SDSP_ERR_PROCESSING;
    }
}

// Whether `cfg` at `sample_rate` takes the default key path's block-folded HPCP frame energies
// (include/stratum_hip_debug.h): the parity tests then compare key_confidence / key_clarity with
// the oracle within the north star's tolerance, and every other configuration bit for bit.
int32_t sdsp_debug_key_energy_blocked(const sdsp_config* cfg, uint32_t sample_rate) {
    if (!cfg || sample_rate == 0) return -1;
    return key_energy_blocked(*cfg, sample_rate) ? 1 : 0;
}

// Per track of the last sdsp_analyze_batch_device / sdsp_analyze_audio call on `device`: 1 where
// its key vote was near an energy-dependent decision and the track was analysed again exactly.
int32_t sdsp_debug_last_key_near(int32_t device, uint8_t* out, uint64_t n) {
    try {
        DeviceCtx& d = device_ctx(device);
        std::lock_guard<std::mutex> lk(d.mu);
        for (uint64_t i = 0; i < n; i++) out[i] = i < d.last_near.size() ? d.last_near[(size_t)i] : 0;
        return SDSP_OK;
    } catch (const std::exception&) {
        return SDSP_ERR_PROCESSING;
    }
}

// Host buffers: chunks of whole tracks (up to SDSP_BATCH_CHUNK_TRACKS tracks, default
// 512, and about 8 GB) pulled from a shared counter by one worker per device; per device a copier
// thread stages the next chunk into the second of two HBM slots (its own stream, completion
// signalled by an event the engine's stream waits on) while the device analyses the current one.
// The queue itself is batch_sched.hpp (host-only, tested with fake devices).
int32_t sdsp_analyze_batch(const float* const* tracks, const uint64_t* lens, uint64_t n_tracks, uint32_t sample_rate,
                           const sdsp_config* cfg, uint32_t device_mask, sdsp_result* outs) {
    std::vector<int> devs;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        for (uint64_t i = 0; i < n_tracks; i++) {
            std::memset(&outs[i], 0, sizeof(outs[i]));
            outs[i].status = SDSP_ERR_PROCESSING;
            std::snprintf(outs[i].error_message, sizeof outs[i].error_message, "Processing error: no HIP device");
        }
        return SDSP_ERR_PROCESSING;
    }
    devs = device_list_override(ndev);
    if (devs.empty())
        for (int d = 0; d < ndev && d < 32; d++)
            if (device_mask == 0 ? d == 0 : ((device_mask >> d) & 1u)) devs.push_back(d);
    if (devs.empty()) devs.push_back(0);
    uint64_t max_tracks = 512;
    if (const uint64_t t = test_hooks().batch_chunk_tracks.load()) max_tracks = t;  // sdsp_debug_set_schedule
    const std::vector<uint64_t> cb = plan_chunks(lens, n_tracks, max_tracks, (uint64_t)2 << 30 /* 8 GB of f32 */);
    // test hook (sdsp_debug_set_test_hooks): the chunk whose analysis throws (the per-chunk failure path)
#ifdef SDSP_TEST_HOOKS
    const long fail_chunk = test_hooks().fail_chunk.load();
#endif
    const size_t n_chunks = cb.size() - 1;
    // every result starts as an error; run_device overwrites the tracks it analyses
    auto mark_failed = [&](size_t c, const std::string& what) {
        for (uint64_t i = cb[c]; i < cb[c + 1]; i++) {
            std::memset(&outs[i], 0, sizeof(outs[i]));
            outs[i].status = SDSP_ERR_PROCESSING;
            std::snprintf(outs[i].error_message, sizeof outs[i].error_message, "Processing error: %s", what.c_str());
        }
    };
    for (size_t c = 0; c < n_chunks; c++) mark_failed(c, "track not analysed");
    std::vector<DeviceStage*> stg;
    std::vector<ChunkDevice> cds;
    for (int dev : devs) {
        stg.push_back(stage_acquire(dev));
        DeviceStage* ds = stg.back();
        ChunkDevice cd;
        cd.stage = [ds, &cb, tracks, lens](int s, size_t c) {
            SDSP_HIP_CHECK(hipSetDevice(ds->dev));
            if (!ds->copy) SDSP_HIP_CHECK(hipStreamCreateWithFlags(&ds->copy, hipStreamNonBlocking));
            Slot& sl = ds->slot[s];
            if (!sl.ready) SDSP_HIP_CHECK(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
            uint64_t tot = 0;
            for (uint64_t i = cb[c]; i < cb[c + 1]; i++) tot += lens[i];
            if (sl.cap < tot) {
                if (sl.d) SDSP_HIP_CHECK(hipFree(sl.d));
                sl.d = nullptr;
                sl.cap = 0;
                const uint64_t want = std::max<uint64_t>(tot + tot / 8, 1);  // grow-only, with slack
                SDSP_HIP_CHECK(hipMalloc(&sl.d, want * sizeof(float)));
                note_alloc(want * sizeof(float));
                sl.cap = want;
            }
            uint64_t o = 0;
            for (uint64_t i = cb[c]; i < cb[c + 1]; i++) {
                if (lens[i])
                    SDSP_HIP_CHECK(hipMemcpyAsync(sl.d + o, tracks[i], lens[i] * sizeof(float), hipMemcpyHostToDevice,
                                                  ds->copy));
                o += lens[i];
            }
            SDSP_HIP_CHECK(hipEventRecord(sl.ready, ds->copy));
        };
#ifdef SDSP_TEST_HOOKS
        cd.analyze = [ds, &cb, lens, sample_rate, cfg, outs, fail_chunk](int s, size_t c) {
            if ((long)c == fail_chunk) throw HipError("injected chunk failure (test hook)");
#else
        cd.analyze = [ds, &cb, lens, sample_rate, cfg, outs](int s, size_t c) {  // (no failure injection)
#endif
            const uint64_t a = cb[c], b = cb[c + 1];
            std::vector<uint64_t> off(b - a), ln(b - a);
            uint64_t tot = 0;
            for (uint64_t i = a; i < b; i++) {
                off[i - a] = tot;
                ln[i - a] = lens[i];
                tot += lens[i];
            }
            run_device(ds->dev, ds->slot[s].d, off.data(), ln.data(), b - a, sample_rate, cfg, nullptr, outs + a,
                       SDSP_STAGES_FULL, ds->slot[s].ready);
        };
        cd.drain = [ds]() {  // after a failed chunk: nothing may still read the slot it reuses
            // the engine's own streams and this stage's copy stream, never the caller's streams
            SDSP_HIP_CHECK(hipSetDevice(ds->dev));
            DeviceCtx& c = device_ctx(ds->dev);
            {
                std::lock_guard<std::mutex> lk(c.mu);
                for (hipStream_t s : c.own) SDSP_HIP_CHECK(hipStreamSynchronize(s));
            }
            if (ds->copy) SDSP_HIP_CHECK(hipStreamSynchronize(ds->copy));
        };
        cds.push_back(cd);
    }
    const size_t failed = run_chunked(n_chunks, cds, [&](size_t c, const std::string& what) {
        std::fprintf(stderr, "sdsp_analyze_batch: %s\n", what.c_str());
        mark_failed(c, what);
    });
    for (DeviceStage* ds : stg) stage_release(ds);
    return failed ? SDSP_ERR_PROCESSING : SDSP_OK;
}

int32_t sdsp_analyze_audio(const float* samples, uint64_t n_samples, uint32_t sample_rate, const sdsp_config* cfg,
                           sdsp_result* out, char* err, uint64_t errlen) {
    std::memset(out, 0, sizeof(*out));
    if (n_samples == 0 || sample_rate == 0) {
        const char* m = n_samples == 0 ? "Invalid input: Empty audio samples" : "Invalid input: Invalid sample rate";
        if (err && errlen) std::snprintf(err, (size_t)errlen, "%s", m);
        out->status = SDSP_ERR_INVALID_INPUT;
        return SDSP_ERR_INVALID_INPUT;
    }
    // one track: staged into a context buffer on the engine's stream under the context lock (no
    // copy stream, copier thread or staging allocation per call); device 0, as the batch's
    // default mask
    int32_t rc = SDSP_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        out->status = SDSP_ERR_PROCESSING;
        std::snprintf(out->error_message, sizeof out->error_message, "Processing error: no HIP device");
    } else {
        try {
            DeviceCtx& d = device_ctx(0);
            std::lock_guard<std::mutex> lk(d.mu);
            SDSP_HIP_CHECK(hipSetDevice(0));
            DevBuf& in = d.buf("api.track");
            in.ensure(n_samples * sizeof(float));
            SDSP_HIP_CHECK(hipMemcpyAsync(in.p, samples, n_samples * sizeof(float), hipMemcpyHostToDevice, d.stream));
            const uint64_t off = 0;
            rc = run_locked(d, in.as<float>(), &off, &n_samples, 1, sample_rate, cfg, nullptr, out, SDSP_STAGES_FULL,
                            nullptr);
        } catch (const std::exception& e) {
            std::memset(out, 0, sizeof(*out));
            out->status = SDSP_ERR_PROCESSING;
            std::snprintf(out->error_message, sizeof out->error_message, "Processing error: %s", e.what());
        }
    }
    if (rc != SDSP_OK && out->status == SDSP_OK) out->status = rc;
    if (out->status != SDSP_OK) {
        if (err && errlen) std::snprintf(err, (size_t)errlen, "%s", out->error_message);
        const int32_t s = out->status;
        sdsp_result_free(out);
        std::memset(out, 0, sizeof(*out));
        out->status = s;
        return s;
    }
    return SDSP_OK;
}

int32_t sdsp_generate_synthetic(float* d_out, uint64_t n_tracks, uint64_t len, uint32_t sample_rate, uint64_t seed0,
                                int32_t bpm_mode, int32_t device, void* stream, float* bpm_out, int32_t* key_out) {
    try {
        DeviceCtx& d = device_ctx(device);
        std::lock_guard<std::mutex> lk(d.mu);
        SDSP_HIP_CHECK(hipSetDevice(device));
        std::vector<float> bpm((size_t)n_tracks);
        std::vector<int> key((size_t)n_tracks);
        for (uint64_t i = 0; i < n_tracks; i++) {
            uint64_t x = 0x5EED0000ull + seed0 + i;
            auto next = [&]() {  // splitmix64
                x += 0x9E3779B97F4A7C15ull;
                uint64_t z = x;
                z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                return z ^ (z >> 31);
            };
            float b;
            if (bpm_mode == 1) {  // config 5: thirds in [55,80], [170,200], [80,170]
                const int third = (int)(i % 3);
                const uint64_t r = next();
                if (third == 0)
                    b = 55.0f + 0.5f * (float)(r % 51);
                else if (third == 1)
                    b = 170.0f + 0.5f * (float)(r % 61);
                else
                    b = 80.0f + 0.5f * (float)(r % 181);
            } else {
                b = 70.0f + 0.5f * (float)(next() % 221);
            }
            bpm[(size_t)i] = b;
            key[(size_t)i] = (int)(next() % 24);
        }
        if (bpm_out) std::memcpy(bpm_out, bpm.data(), bpm.size() * sizeof(float));
        if (key_out) std::memcpy(key_out, key.data(), key.size() * sizeof(int));
        hipStream_t st = stream ? (hipStream_t)stream : d.stream;
        DevBuf& db = d.buf("synth.bpm");
        db.ensure(bpm.size() * 4 + 16);
        DevBuf& dk = d.buf("synth.key");
        dk.ensure(key.size() * 4 + 16);
        DevBuf& dp = d.buf("synth.peak");
        dp.ensure(key.size() * 4 + 16);
        SDSP_HIP_CHECK(hipMemcpyAsync(db.p, bpm.data(), bpm.size() * 4, hipMemcpyHostToDevice, st));
        SDSP_HIP_CHECK(hipMemcpyAsync(dk.p, key.data(), key.size() * 4, hipMemcpyHostToDevice, st));
        launch_synth(d_out, n_tracks, len, sample_rate, db.as<float>(), dk.as<int>(), seed0, st);
        launch_synth_normalize(d_out, n_tracks, len, dp.as<unsigned int>(), st);
        SDSP_HIP_CHECK(hipGetLastError());
        SDSP_HIP_CHECK(hipStreamSynchronize(st));
        return SDSP_OK;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "sdsp_generate_synthetic: %s\n", e.what());
        return SDSP_ERR_PROCESSING;
    }
}

}  // extern "C"
