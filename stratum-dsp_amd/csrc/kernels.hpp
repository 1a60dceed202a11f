// kernels.hpp — parameter structs shared between the kernels and the pipeline, and the host
// launchers each kernel file exports (kernels are launched only from their own TU).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdsp_device.hpp"

namespace sdsp {

constexpr int NVAR = 5;  // novelty variants: full, low, mid, high, mel

// ---- k_features ----
// the mel plans of one 8-bin chunk: per bin j, bits 4j..4j+1 = nflush (<= 3), bit 4j+2 = s0,
// bit 4j+3 = s1; w0 / w1 as MelPlan (0: no contribution)
struct MelChunk {
    uint32_t bits;
    float w0[8], w1[8];
    float bf[8];  // (float) b of the chunk's bins, the HFC weights (every chunk, mel or not)
};
struct FeatParams {
    int B;             // bins per frame (nfft/2+1)
    int stride;        // row stride of mags
    int K;             // SuperFlux max-filter half width
    int bs[4], be[4];  // band [start, end) for v = full, low, mid, high
    int band_on[4];    // variant enabled (full always)
    int n_mels;
    // per 8-bin chunk of k_features<8, 16, 4> (host-built, feat_chunk_flags): bits 0-1 the band
    // of every bin of the chunk, bit 2 = FT_CHUNK_FAST (one band, no band-edge clipping of the
    // SuperFlux window, no mel work, full chunk)
    const int* chunk_flags;
    // FT_CHUNK_MEL chunks (bit 3: as FT_CHUNK_FAST, but with mel work): the chunk's 8 mel plans
    // packed (MelChunk), indexed by chunk; its bf (HFC weights) is read by every fast chunk
    const MelChunk* mel_chunks;
};
// FT_CHUNK_MELREG (with FT_CHUNK_MEL): every bin's w0 goes to accumulator 0 and w1 to 1 (or is 0)
constexpr int FT_CHUNK_FAST = 4, FT_CHUNK_MEL = 8, FT_CHUNK_MELREG = 16;
// per-bin mel accumulation plan (k_features): flush `nflush` finished mels before the bin,
// then, in the reference's contribution order, add L*w0 to accumulator s0 and L*w1 to s1
// (accumulator 0 = mel mA, 1 = mel mA+1; w = 0 means no contribution)
struct MelPlan {
    int nflush;
    int s0, s1;
    float w0, w1;
};
#ifndef SDSP_PK_CH
#define SDSP_PK_CH 16384
#endif
constexpr int PK_CH = SDSP_PK_CH;  // samples per k_peak_abs workgroup
constexpr int FT_FRAMES = 256;
// frames per k_features tile: lane 0 of each wave is a helper that computes the normalised
// magnitudes of the frame before the wave's first (k_features.hip)
constexpr int FT_STEP = FT_FRAMES - FT_FRAMES / 64;
// Where k_features finds frame f of item k: row (f even ? A : B) r0 + (f >> 1) * step, with
// rB0 = rowB0[k] or rowA0[k] + offB.  Compact spectrogram: A = B, rowA0 = frame prefix, offB = 1,
// steps 2.  The escalation hops reuse the hop-512 rows: hop 1024 frame v is hop-512 frame 2v;
// hop 256 frame 2u is hop-512 frame u (the odd hop-256 frames are computed on their own).
struct RowMap {
    const float *magsA, *magsB, *fmaxA, *fmaxB;
    const uint64_t *rowA0, *rowB0;
    int offB, stepA, stepB;
};
constexpr int FT_KMAX = 8;
constexpr int FT_MELMAX = 48;

// ---- k_novelty ----
struct NovParams {
    float ws, we, wh, wsum;
    int lmw, smw;
    int band_on[4];
};

// ---- k_tempo ----
struct FftTgParams {
    int P;
    int b_lo, K;
    float fres;
    int lds;
};
struct SelParams {
    float min_bpm, max_bpm, ac_tol;
    float w[NVAR];
    int present[NVAR];
    int seed_only;
    float support_thr, bonus;
    int bonus_on;
    int top_n;
    int NB;
    int gate;
    int gate_top_n;
    float gate_tol;
};
struct TempoEst {
    float bpm, conf;
    int agree;
    int ok;
    int n_cands;
    int ambiguous, trap_low, trap_high;
};
struct MrParams {
    float min_bpm, max_bpm, tol, w512, w256, w1024, dt, margin_thr;
    int human_prior, top_k, band;
    int sr, hop512;
    int own512;  // 1: the hop-512 lists / novelty are the escalation's own pass (item order), else the base pass's (track order)
};

// debug_track_id diagnostics (src/lib.rs:461-487, 547-573, multi_resolution.rs:707-860): what
// k_multires decided, written only when a record buffer is passed
struct MrDbg {
    int fd, fu, tf;                   // fold-down / fold-up / triplet-family switch taken
    float fd_from, fd_to, fd_ratio;   // fold-down: best -> half, support ratio
    int fd_a0, fd_a1;                 //   hop agreement before / after
    float fu_from, fu_to, fu_ratio;   // fold-up: best -> double
    int fu_a0, fu_a1;
    float tf_from, tf_to;             // triplet family: current -> chosen
    float tf_sup0, tf_sup1;           //   support / best family support, current and chosen
    float tf_al0, tf_al1;             //   beat-contrast alignment, current and chosen
    int tf_label;                     //   family factor index: T, 3/2, 2/3, 4/3, 3/4
    float rel;                        // acceptance (src/lib.rs:515-545)
    int fam, forbid, better;
};
// k_key_vote's final score table and the weighted pitch-class summary (src/lib.rs:1471-1538)
struct KeyDbg {
    float tab[24];  // scores, descending
    int order[24];  // key index (0-11 major, 12-23 minor) of each
    int key;        // chosen key
    float agg[12];  // weighted pitch-class sums over the slice, normalised by their sum
    int frames, used;
};

// ---- k_beat ----
struct BeatOut {
    int n_beats, n_down;
    float stability;
    int ok;
};

// ---- k_key ----
constexpr int HP_KMAX = 32;
constexpr int HP_FRAMES = 256;  // frames per k_hpcp workgroup
constexpr int HP_HMAX = 8;
struct HarmEntry {
    int state;
    int tc[3];
    float wt[3];
    float hw;
};
struct HpcpParams {
    int B, stride, pk_lo, pk_hi;
    int K;
    int hmax;
    float p;
};
struct KeyParams {
    int weighting;
    float min_tonal, tonal_pow, energy_pow;
    int seg_voting;
    int seg_len, seg_hop;
    float min_clarity;
    // opt-in branches (src/lib.rs:1200-1470)
    float sharpen;             // chroma_sharpening_power (applied when > 1)
    int edge_trim;             // enable_key_edge_trim
    float edge_frac;           // key_edge_trim_fraction
    int ensemble;              // enable_key_ensemble
    float kk_w, tp_w;          // key_ensemble_{kk,temperley}_weight
    int tset;                  // key_template_set (0 K-K, 1 Temperley)
    int mh_on, mh_bonus;       // mode heuristic || minor bonus; minor bonus
    float mh_margin, mh_flip;  // third-ratio margin; flip ratio (0 unless the heuristic is on)
    float mh_bonus_w;          // leading-tone bonus weight
    int ms_on, ms_n, ms_hop, ms_nw;  // multi-scale: enabled, #lengths (<= 8), hop, #weights
    float ms_min_cl;
    int ms_len[8];
    float ms_w[8];
    // the default key path's block-folded frame energies are in use: report in
    // KeyOut::near whether a discrete decision downstream of the energies is within a margin the
    // re-association could cross, so the host reruns that track with the sequential fold
    int near_check;
    // near_check margins: 0 the rigorous certificate (the per-frame energy bounds k_hpcp_band
    // writes, carried through the weights, raw scores, clarities and the vote, with the fixed
    // round-5 margins below as floors); 1 the fixed margins alone (sdsp_debug_set_key_cert, for A/B)
    int cert_fixed;
};
// near-decision margins (k_key_vote, KeyParams::near_check): a segment clarity within
// KV_NEAR_CLARITY of its gate, a final (best - second) / best below KV_NEAR_CONF, or a weight sum
// within KV_NEAR_REL of the 1e-12 fallback threshold.  The re-association moves clarities by
// <= 1e-6 and relative score gaps by <= 1e-6 on every track measured (profiles/r05_key_scale.jsonl),
// so the margins hold a factor of 100.
constexpr float KV_NEAR_CLARITY = 1e-4f, KV_NEAR_CONF = 1e-4f, KV_NEAR_REL = 1e-3f;
// k_key_vote's segment scratch row (floats): 24 sorted, 24 order, clarity, used, cw, wsum, avg[12];
// then the certificate's per-key partial-sum totals [64, 88) and energy sensitivities [88, 112)
// (the clarity stage replaces [64, 88) by the post-bonus score bounds), [112] the clarity bound
constexpr int KV_ROW = 128;
// KeyOut::near bits: which decision was within its margin
constexpr int KV_NEAR_ARGMAX = 1, KV_NEAR_GATE = 2, KV_NEAR_FINAL = 4, KV_NEAR_WSUM = 8;
// (16: a frame weight or energy outside the certificate's range: underflow, or no usable bound)
constexpr int KV_NEAR_RANGE = 16;
struct KeyOut {
    int mode, tonic;
    float conf, clarity;
    int ok;
    int used_segments;
    int weights_used;
    int near;  // near_check only: KV_NEAR_* bits of the energy-dependent decisions within their margin (rerun exactly)
};

// ---- k_chroma (opt-in chroma front-ends) ----
struct TuningParams {
    int stride, lo, hi, step, chf;  // band bins [lo, hi]; sampled-frame step; frames per LDS batch
    float fres, thr, lim;           // bin spacing; peak-relative threshold; |offset| clamp
};
struct ChromaBin {
    int a, b;  // k_chroma<0>: primary class; k_chroma<1>: lo, hi semitone bins (a = -1: none)
    float w0, w1, w2;
};
struct ChromaParams {
    int B, stride, lo, hi;  // bins per row, row stride, mapped bin range [lo, hi]
    int soft, gate_small;   // soft mapping; tuning used only if |offset| > 1e-6
    int n_log, log_off, bmin;  // log-frequency: semitone bins, pitch-class offset, first semitone
    float fres, sigma;
};
struct HpcpXParams {
    int B, stride;
    int pk_lo, pk_hi, bk_lo, bk_hi;  // main / bass candidate bins
    int K, KB, hmax;
    int half, rp, rp_mask, rx, rx_mask;  // whitening half width (0 = off) and LDS ring sizes
    int bass, main_ok, bass_ok;
    float p, fres, fmin, fmax, bfmin, bfmax, decay, sigma, bw;
};

struct KeyHpssParams {
    int B, stride, bin0, nb;  // bins per row; row stride; median band [bin0, bin0 + nb)
    int step, tm, fm;         // frame step; time / frequency margins (<= 16)
    float p;                  // mask power (>= 1)
};
constexpr int KH_TILE_FRAMES = 16, KH_TILE_BINS = 64, KH_APPLY_FRAMES = 8;  // k_key_hpss_* tiling

// ---- k_hpss (hpss_decompose, hpss.rs:71-281) ----
struct HpssParams {
    int B, stride, m;  // bins per row, row stride, median half width (hpss_margin, <= 16)
};
struct HpssLaunch {
    HpssParams P;
    const float* orig;           // the spectrogram (round 0 input, re-partitioned every round)
    const uint64_t* orig_row0;   // per item: first row of its frames in `orig`
    float* h[2];                 // ping-pong harmonic buffers
    float* p[2];                 // ping-pong percussive buffers (the result ends in p[0])
    const uint64_t* row0;        // per item: first row in h / p (== fpfx: compact)
    const uint64_t* fpfx;        // frame prefix over the items
    const uint64_t* vtile_pfx;   // k_hpss_round tiles: ceil(F / 32) * ceil(B / 256) per item
    uint64_t n_vtiles;
    int* last_it;                // per item: last round run (init 9)
    unsigned int* change;        // per item: the round's largest change (f32 bits)
    int n_items;
};
constexpr int HPSS_VM_FRAMES = 32, HPSS_COLS = 256, HPSS_ROW_FRAMES = 256;

// ---- k_legacy (estimate_bpm_with_guardrails / estimate_bpm, period/mod.rs:196-404) ----
struct LegacyParams {
    int sr, hop;
    float min_bpm, max_bpm, res;
    int guard;   // enable_legacy_bpm_guardrails
    float g[7];  // clamp_sane'd guardrails: preferred min/max, soft min/max, mul preferred/soft/extreme
};
struct LegacyOut {
    int ok;  // 1 estimate, 0 none, -1 "Signal too short for autocorrelation", -2 scratch too small
    float bpm, conf;
    int agree;
};
constexpr int LG_COMB_MAX = 2048, LG_AC_MAX = 512;  // comb candidates; autocorrelation peaks

// ---- launchers ----
// launch_stft, stft_strips, stft_slide_ok: sdsp_runtime.hpp
// chunk_bits: n_chunks words of scratch (each k_peak_abs workgroup's maximum)
void launch_peak_gain(const float* x, const uint64_t* in_off, const uint64_t* n_raw, const uint64_t* chunk_pfx, int T,
                      uint64_t n_chunks, unsigned int* chunk_bits, unsigned int* peak_bits, float target, int enable,
                      float* gain, hipStream_t st);
// RMS / LUFS normalization constants, computed on the host (normalization.rs:119-158, 325-470)
struct LoudnessParams {
    int method;          // 1 RMS, 2 LUFS
    float target_rms;    // 10^((target_lufs + 3 - headroom) / 20)
    float target_peak;   // 10^((0 - headroom) / 20)
    float target_lufs;   // -14
    float gate;          // 10^((-70 + 0.691) / 10)
    int64_t block;       // 400-ms block, samples
    float b0, b1, b2, a1, a2;  // K-weighting biquad, normalised by a0
};
void launch_loudness_gain(const float* x, const uint64_t* in_off, const uint64_t* n_raw, const uint64_t* chunk_pfx,
                          int T, uint64_t n_chunks, unsigned int* chunk_bits, unsigned int* peak_bits,
                          const LoudnessParams& P, float* gain, int* status, hipStream_t st);
void launch_frame_rms(const float* x, const uint64_t* src_off, const float* gain, const uint64_t* n_len,
                      const uint64_t* frame_pfx, int T, uint64_t total, int fs, int hop, float* rms, hipStream_t st, bool per_frame_kernel = false);
// base_pfx / stride: trim frame f of track t at rms[base_pfx[t] + f * stride] (default: frame_pfx, 1)
void launch_trim(const float* rms, const uint64_t* frame_pfx, int T, const uint64_t* n_raw, int hop, float thr,
                 uint64_t min_frames, int enable, uint64_t* trim_start, uint64_t* trim_end, hipStream_t st,
                 const uint64_t* base_pfx = nullptr, int stride = 1);
// the energy pass's frame RMS (fs, hop) of the trimmed tracks from `raw`, the same framing of the
// raw tracks (k_rms_gather), frame j of track i at raw[raw_base[i] + j]; frames the trimmed end
// cuts short are computed from the samples
void launch_frame_rms_from_raw(const float* raw, const uint64_t* raw_base, const float* x, const uint64_t* src_off,
                               const float* gain, const uint64_t* n_trim, const uint64_t* frame_pfx, int T, uint64_t total,
                               int fs, int hop, float* rms, hipStream_t st);
void launch_energy_onsets(const float* rms, const uint64_t* frame_pfx, const uint64_t* n_trim, int hop, float factor,
                          uint32_t* out, const uint64_t* out_off, int* out_n, int T, hipStream_t st);
void launch_flux_onsets(const float* sfo, const float* hfc, const float* hpe, float* scratch, const uint64_t* frame_pfx,
                        const uint64_t* n_trim, int hop, float pct, uint32_t* out, const uint64_t* out_off,
                        int* out_n, int T, hipStream_t st);
void launch_consensus(const uint32_t* energy, const uint64_t* e_off, const int* e_n, const uint32_t* flux_on,
                      const uint64_t* f_off, const int* f_n, uint64_t kind_stride, int T, uint32_t tol, int enable,
                      const int* has_mags, uint32_t* chosen, const uint64_t* c_off, int* c_n, uint32_t* scratch,
                      hipStream_t st, int hpss = 0);
void launch_features(const RowMap& mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx,
                     int T, uint64_t n_tiles, const FeatParams& P, const MelPlan* mel, float* E, float* H, float* SFX,
                     float* SFO, float* MEL, uint64_t total, hipStream_t st);
void launch_novelty(const float* E, const float* H, const float* SFX, const uint64_t* frame_pfx, int T, uint64_t total,
                    const NovParams& P, float* scratch, float* nov, float* nov_sum, const float* MEL, int n_mels,
                    int mel_k, bool mel_on, unsigned int* mel_max, hipStream_t st);
void launch_fft_tempogram(const int* items, int n_items, int T, const float* nov, const float* nov_sum,
                          const uint64_t* frame_pfx, uint64_t total, const FftTgParams& P, const cx* tw, const cx* rt,
                          cx* gscratch, const uint64_t* out_off, float* out_bpm, float* out_pow, hipStream_t st);
void launch_acf_tempogram(const int* items, int n_items, const float* nov, const uint64_t* frame_pfx, uint64_t total,
                          const float* bpm_grid, const int* lag_grid, int NB, float* out_bpm, float* out_str,
                          hipStream_t st);
void launch_tempo_select(int n_items, const int* active, const float* fft_bpm, const float* fft_pow, const uint64_t* fft_off,
                         const int* fft_k, const float* acf_bpm, const float* acf_str, const uint64_t* acf_off,
                         const SelParams& P, TempoEst* est, float* cand, int cand_cap, hipStream_t st);
void launch_multires(const int* tracks, int n_items, const float* c256, const int* n256, const float* c512,
                     const int* n512, const float* c1024, const int* n1024, int cap256, int cap512, int cap1024,
                     const TempoEst* base_est, const float* nov512, const uint64_t* fpfx512, const MrParams& P,
                     TempoEst* mr_est, int* used, float* final_bpm, float* final_conf, hipStream_t st, MrDbg* dbg = nullptr);
void launch_beat(const int* tracks, int n_items, const uint32_t* onsets, const uint64_t* on_off, const int* on_n,
                 uint32_t sr, const float* bpm, const float* conf, float* scratch, const uint64_t* beat_off,
                 const int* beat_cap, float* beats, float* downs, BeatOut* out, hipStream_t st);
// dense beat/downbeat lists: pfx has 2 (n + 1) entries (beats, then downbeats)
void launch_beat_compact(int n, const BeatOut* out, const uint64_t* beat_off, const float* beats, const float* downs,
                         uint64_t* pfx, float* cb, float* cd, hipStream_t st);
void launch_mask(float* mags, int stride, int B, const uint64_t* frame_pfx, const int* tracks, int n_items, int margin,
                 float power, hipStream_t st, bool smooth_only = false);
void launch_tuning(const float* mags, const uint64_t* frame_pfx, const int* tracks, int n_items, const TuningParams& P,
                   float* out, hipStream_t st);
void launch_chroma(int mode, const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                   int n_items, uint64_t n_tiles, const ChromaParams& P, const float* tuning, float* chroma,
                   float* energy, hipStream_t st);
void launch_hpcp_x(const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                   int n_items, uint64_t n_tiles, const HpcpXParams& P, const float* tuning, float* chroma,
                   float* energy, hipStream_t st);
void launch_key_hpss(float* mags, const uint64_t* frame_pfx, const uint64_t* mtile_pfx, uint64_t n_mtiles,
                     const uint64_t* atile_pfx, uint64_t n_atiles, const uint64_t* mask_off, const int* tracks,
                     int n_items, const KeyHpssParams& P, float* mask, hipStream_t st);
void launch_hpss(const HpssLaunch& L, hipStream_t st);
void launch_legacy(const uint32_t* onsets, const uint64_t* on_off, const int* on_n, int n_items, const uint64_t* scr_off,
                   const uint64_t* scr_cap, cx* scratch, const cx* tw, int tw_M, const LegacyParams& P, LegacyOut* out,
                   hipStream_t st);
void launch_hpss_rows(const float* p, const uint64_t* row0, const uint64_t* fpfx, const uint64_t* tile_pfx,
                      uint64_t n_tiles, int n_items, int stride, int B, float* energy, float* fmax, hipStream_t st);
void launch_beat_sync(const int* tracks, int n_items, const uint64_t* frame_pfx, const float* fchroma,
                      const float* fenergy, const float* beats, const uint64_t* beat_off, const uint64_t* row_pfx,
                      float fd, float* chroma, float* energy, hipStream_t st);
// the default key path's band-limited mask + block energy sums and the HPCP that reads them
// (k_key.hip k_mask_rp / k_hpcp_band; only for margin 12, power 2)
bool mask_band_ok(int margin, float power);
void launch_mask_band(float* mags, int stride, int B, const uint64_t* frame_pfx, const int* tracks, int n_items,
                      float power, int st_lo, int st_hi, float* part, uint64_t total, hipStream_t st,
                      bool outside = false);
void launch_hpcp_band(const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                      int n_items, uint64_t n_tiles, const HpcpParams& P, const HarmEntry* harm, const float* part,
                      uint64_t total, float* chroma, float* energy, float* edel, hipStream_t st);
void launch_hpcp(const float* mags, const uint64_t* frame_pfx, const uint64_t* tile_pfx, const int* tracks,
                 int n_items, uint64_t n_tiles, const HpcpParams& P, const HarmEntry* harm, float* chroma,
                 float* energy, hipStream_t st);
void launch_key_vote(const int* tracks, int n_items, const uint64_t* frame_pfx, float* chroma_raw,
                     const float* energy, float* chroma_s, float* weights, float* seg_scratch, const uint64_t* seg_off,
                     const float* tmpl, const KeyParams& P, KeyOut* out, hipStream_t st, KeyDbg* dbg = nullptr,
                     const float* edel = nullptr, float* wdel = nullptr, bool alone = false);
void launch_synth(float* out, uint64_t n_tracks, uint64_t len, uint32_t sr, const float* bpm, const int* key,
                  uint64_t seed0, hipStream_t st);
void launch_synth_normalize(float* out, uint64_t n_tracks, uint64_t len, unsigned int* peak_bits, hipStream_t st);

}  // namespace sdsp
