// runtime.hip — device contexts, FFT tables, C ABI housekeeping (config defaults, result
// ownership, version) and stage probes.  The analyze pipeline itself is in pipeline.hip.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "../../include/sdsp_fft_spec.h"
#include "../../include/stratum_hip_debug.h"
#include "kernels.hpp"
#include "sdsp_runtime.hpp"

namespace sdsp {

static std::atomic<uint64_t> g_alloc_n{0}, g_alloc_bytes{0};
void note_alloc(size_t bytes) {
    g_alloc_n++;
    g_alloc_bytes += bytes;
}

static std::mutex g_ctx_mu;
static std::map<int, std::unique_ptr<DeviceCtx>> g_ctx;

TestHooks& test_hooks() {
    static TestHooks h;
    return h;
}
std::vector<int> test_hooks_devices() {
    TestHooks& h = test_hooks();
    std::lock_guard<std::mutex> lk(h.mu);
    return h.devices;
}

DeviceCtx& device_ctx(int device) {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto& c = g_ctx[device];
    if (!c) {
        c.reset(new DeviceCtx());
        c->device = device;
        SDSP_HIP_CHECK(hipSetDevice(device));
        // The tempo path (main stream) is the critical path and is made of short, latency-bound
        // kernels; the key path (stream2) is long bandwidth-bound kernels.  The main stream gets
        // the higher priority so its workgroups are dispatched ahead of the key stream's
        // (measured in round 2: the key stream first, equal priorities and CU-masked streams were
        // all slower end to end).
        int lo = 0, hi = 0;
        SDSP_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        SDSP_HIP_CHECK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
        SDSP_HIP_CHECK(hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, lo));
        // k_key_vote (one 256-thread workgroup per track: latency-bound, a few waves per CU) runs on
        // its own stream so the next sub-batch's 8192-point STFT and mask need not wait behind it
        SDSP_HIP_CHECK(hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, lo));
        SDSP_HIP_CHECK(hipEventCreateWithFlags(&c->vote_done, hipEventDisableTiming));
        for (hipStream_t s : {c->stream, c->stream2, c->stream3}) c->own.push_back(s);
    }
    return *c;
}

FftTables& DeviceCtx::tables(int N, bool with_window) {
    auto& t = fft[N];
    if (!t) {
        t.reset(new FftTables());
        const int M = N / 2;
        std::vector<float> tw(2 * (size_t)std::max(M, 1)), rt((size_t)N + 2);
        sdsp_fft_twiddles(std::max(M, 1), tw.data());
        sdsp_rfft_twiddles(N, rt.data());
        t->tw.ensure(tw.size() * 4);
        t->rt.ensure(rt.size() * 4);
        SDSP_HIP_CHECK(hipMemcpy(t->tw.p, tw.data(), tw.size() * 4, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(t->rt.p, rt.data(), rt.size() * 4, hipMemcpyHostToDevice));
    }
    if (with_window && !t->window.p) {
        std::vector<float> w((size_t)N);
        // extractor.rs:318-323, times 2^32 (exact): the STFT section of sdsp_fft_spec.h scales the
        // windowed frame so |X|^2 stays clear of the subnormal range, and |X| carries 2^-33
        for (int i = 0; i < N; i++) w[(size_t)i] = sdsp_hann_f32(i, N) * 0x1p32f;
        t->window.ensure(w.size() * 4);
        SDSP_HIP_CHECK(hipMemcpy(t->window.p, w.data(), w.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> tw(2 * (size_t)(N / 2)), rt((size_t)N + 2), a, b;
        sdsp_fft_twiddles(N / 2, tw.data());
        sdsp_rfft_twiddles(N, rt.data());
        if (stft_tuned(N)) {  // k_stft_gen reads tw / rt as they are
            stft_tables(N, tw, rt, &a, &b);
            t->stft_tw.ensure(a.size() * 4);
            t->stft_rt.ensure(b.size() * 4);
            SDSP_HIP_CHECK(hipMemcpy(t->stft_tw.p, a.data(), a.size() * 4, hipMemcpyHostToDevice));
            SDSP_HIP_CHECK(hipMemcpy(t->stft_rt.p, b.data(), b.size() * 4, hipMemcpyHostToDevice));
        }
    }
    return *t;
}

}  // namespace sdsp

using namespace sdsp;

extern "C" {

// AnalysisConfig::default(), reference src/config.rs:594-744
void sdsp_config_default(sdsp_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->min_amplitude_db = -40.0f;
    c->normalization = SDSP_NORM_PEAK;
    c->enable_normalization = 1;
    c->enable_silence_trimming = 1;
    c->enable_onset_consensus = 1;
    c->onset_threshold_percentile = 0.80f;
    c->onset_consensus_tolerance_ms = 50;
    for (int i = 0; i < 4; i++) c->onset_consensus_weights[i] = 0.25f;
    c->hpss_margin = 10;
    c->enable_legacy_bpm_guardrails = 1;
    c->enable_tempogram_multi_resolution = 1;
    c->tempogram_multi_res_top_k = 25;
    c->tempogram_multi_res_w512 = 0.45f;
    c->tempogram_multi_res_w256 = 0.35f;
    c->tempogram_multi_res_w1024 = 0.20f;
    c->tempogram_multi_res_structural_discount = 0.85f;
    c->tempogram_multi_res_double_time_512_factor = 0.92f;
    c->tempogram_multi_res_margin_threshold = 0.08f;
    c->enable_tempogram_band_fusion = 1;
    c->tempogram_band_low_max_hz = 200.0f;
    c->tempogram_band_mid_max_hz = 2000.0f;
    c->tempogram_band_high_max_hz = 8000.0f;
    c->tempogram_band_w_full = 0.40f;
    c->tempogram_band_w_low = 0.25f;
    c->tempogram_band_w_mid = 0.20f;
    c->tempogram_band_w_high = 0.15f;
    c->tempogram_band_seed_only = 1;
    c->tempogram_band_support_threshold = 0.25f;
    c->tempogram_band_consensus_bonus = 0.08f;
    c->tempogram_novelty_w_spectral = 0.30f;
    c->tempogram_novelty_w_energy = 0.35f;
    c->tempogram_novelty_w_hfc = 0.35f;
    c->tempogram_novelty_local_mean_window = 16;
    c->tempogram_novelty_smooth_window = 5;
    c->debug_top_n = 5;
    c->enable_tempogram_mel_novelty = 1;
    c->tempogram_mel_n_mels = 40;
    c->tempogram_mel_fmin_hz = 30.0f;
    c->tempogram_mel_fmax_hz = 8000.0f;
    c->tempogram_mel_max_filter_bins = 2;
    c->tempogram_mel_weight = 0.15f;
    c->tempogram_superflux_max_filter_bins = 4;
    c->tempogram_candidates_top_n = 10;
    c->legacy_bpm_preferred_min = 72.0f;
    c->legacy_bpm_preferred_max = 168.0f;
    c->legacy_bpm_soft_min = 60.0f;
    c->legacy_bpm_soft_max = 210.0f;
    c->legacy_bpm_conf_mul_preferred = 1.30f;
    c->legacy_bpm_conf_mul_soft = 0.70f;
    c->legacy_bpm_conf_mul_extreme = 0.01f;
    c->min_bpm = 40.0f;
    c->max_bpm = 240.0f;
    c->bpm_resolution = 1.0f;
    c->frame_size = 2048;
    c->hop_size = 512;
    c->center_frequency = 440.0f;
    c->soft_chroma_mapping = 1;
    c->soft_mapping_sigma = 0.5f;
    c->chroma_sharpening_power = 1.0f;
    c->enable_key_spectrogram_time_smoothing = 1;
    c->key_spectrogram_smooth_margin = 12;
    c->enable_key_frame_weighting = 1;
    c->key_min_tonalness = 0.0f;
    c->key_tonalness_power = 2.0f;
    c->key_energy_power = 0.50f;
    c->enable_key_harmonic_mask = 1;
    c->key_harmonic_mask_power = 2.0f;
    c->key_hpss_frame_step = 4;
    c->key_hpss_time_margin = 8;
    c->key_hpss_freq_margin = 8;
    c->key_hpss_mask_power = 2.0f;
    c->enable_key_stft_override = 1;
    c->key_stft_frame_size = 8192;
    c->key_stft_hop_size = 512;
    c->key_template_set = SDSP_TEMPLATES_KRUMHANSL_KESSLER;
    c->key_ensemble_kk_weight = 0.5f;
    c->key_ensemble_temperley_weight = 0.5f;
    c->key_median_segment_length_frames = 480;
    c->key_median_segment_hop_frames = 120;
    c->key_median_min_segments = 3;
    static const uint64_t kMultiScale[3] = {120, 360, 720};
    c->key_multi_scale_lengths = kMultiScale;
    c->key_multi_scale_lengths_len = 3;
    c->key_multi_scale_hop = 60;
    c->key_multi_scale_min_clarity = 0.20f;
    c->key_tuning_max_abs_semitones = 0.08f;
    c->key_tuning_frame_step = 20;
    c->key_tuning_peak_rel_threshold = 0.35f;
    c->key_edge_trim_fraction = 0.15f;
    c->enable_key_segment_voting = 1;
    c->key_segment_len_frames = 1024;
    c->key_segment_hop_frames = 512;
    c->key_segment_min_clarity = 0.20f;
    c->key_mode_third_ratio_margin = 0.00f;
    c->key_mode_flip_min_score_ratio = 0.60f;
    c->enable_key_hpcp = 1;
    c->key_hpcp_peaks_per_frame = 24;
    c->key_hpcp_num_harmonics = 4;
    c->key_hpcp_harmonic_decay = 0.60f;
    c->key_hpcp_mag_power = 0.50f;
    c->key_hpcp_whitening_smooth_bins = 31;
    c->key_hpcp_bass_fmin_hz = 55.0f;
    c->key_hpcp_bass_fmax_hz = 300.0f;
    c->key_hpcp_bass_weight = 0.35f;
    c->key_minor_leading_tone_bonus_weight = 0.2f;
}

const char* sdsp_version(void) { return "stratum-hip 1 gfx950"; }

int32_t sdsp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
int32_t sdsp_device_malloc(int32_t device, uint64_t bytes, void** ptr) {
    if (hipSetDevice(device) != hipSuccess) return SDSP_ERR_PROCESSING;
    return hipMalloc(ptr, bytes ? bytes : 1) == hipSuccess ? SDSP_OK : SDSP_ERR_PROCESSING;
}
int32_t sdsp_device_free(int32_t device, void* ptr) {
    if (hipSetDevice(device) != hipSuccess) return SDSP_ERR_PROCESSING;
    return hipFree(ptr) == hipSuccess ? SDSP_OK : SDSP_ERR_PROCESSING;
}
int32_t sdsp_memcpy_h2d(int32_t device, void* dst, const void* src, uint64_t bytes) {
    if (hipSetDevice(device) != hipSuccess) return SDSP_ERR_PROCESSING;
    return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? SDSP_OK : SDSP_ERR_PROCESSING;
}
int32_t sdsp_memcpy_d2h(int32_t device, void* dst, const void* src, uint64_t bytes) {
    if (hipSetDevice(device) != hipSuccess) return SDSP_ERR_PROCESSING;
    return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? SDSP_OK : SDSP_ERR_PROCESSING;
}
int32_t sdsp_device_synchronize(int32_t device) {
    if (hipSetDevice(device) != hipSuccess) return SDSP_ERR_PROCESSING;
    return hipDeviceSynchronize() == hipSuccess ? SDSP_OK : SDSP_ERR_PROCESSING;
}

void sdsp_result_free(sdsp_result* r) {
    if (!r) return;
    std::free(r->beats);
    std::free(r->downbeats);
    std::free(r->bars);
    for (uint64_t i = 0; i < r->n_warnings; i++) std::free(r->warnings[i]);
    std::free(r->warnings);
    std::free(r->tempogram_candidates);
    r->beats = r->downbeats = r->bars = nullptr;
    r->warnings = nullptr;
    r->tempogram_candidates = nullptr;
    r->n_beats = r->n_downbeats = r->n_bars = r->n_warnings = r->n_tempogram_candidates = 0;
}

int32_t sdsp_last_stage_times(int32_t device, sdsp_stage_times* out) {
    try {
        DeviceCtx& c = device_ctx(device);
        std::lock_guard<std::mutex> lk(c.mu);
        *out = c.last;
        return SDSP_OK;
    } catch (const std::exception&) {
        return SDSP_ERR_PROCESSING;
    }
}

// Kernel probe (tools/stft_probe.py): times `reps` launches of the STFT kernel over n_tracks
// device-resident noise tracks of len samples each (one magnitude buffer, the pipeline's row
// stride), HIP events on the launch stream.  Writes the mean launch time and the algorithmic
// bytes per launch (4 N_in + 4 F (nfft/2+1) per track).
// Test hooks (include/stratum_hip_debug.h).  The library reads no test switch from the
// environment; a test sets these explicitly and resets them with (-1, NULL, 0, 0).
int32_t sdsp_debug_set_test_hooks(int64_t fail_chunk, const int32_t* devices, uint32_t n_devices,
                                  int32_t stft_frame_parallel) {
#ifndef SDSP_TEST_HOOKS
    // the shipping library: failure injection and the device override are compiled only into the
    // test build (lib/libstratum_hip_testhooks.so, -DSDSP_TEST_HOOKS), so nothing can make this
    // library fail a chunk or re-route work; the frame-parallel STFT switch (same results) stays
    if (fail_chunk >= 0 || n_devices > 0) return SDSP_ERR_NOT_IMPLEMENTED;
#endif
    TestHooks& h = test_hooks();
    h.fail_chunk.store((long)fail_chunk);
    h.stft_frame_parallel.store(stft_frame_parallel != 0);
    std::lock_guard<std::mutex> lk(h.mu);
    h.devices.assign(devices ? devices : nullptr, devices ? devices + n_devices : nullptr);
    return SDSP_OK;
}

int32_t sdsp_debug_set_schedule(int32_t serial_streams, int32_t no_key_defer, int32_t no_row_reuse, int32_t host_trace,
                                uint64_t batch_chunk_tracks, double hbm_budget_gb) {
    TestHooks& h = test_hooks();
    h.serial_streams.store(serial_streams != 0);
    h.no_key_defer.store(no_key_defer != 0);
    h.no_row_reuse.store(no_row_reuse != 0);
    h.host_trace.store(host_trace != 0);
    h.batch_chunk_tracks.store(batch_chunk_tracks);
    h.hbm_budget_gb.store(hbm_budget_gb > 0.0 ? hbm_budget_gb : 0.0);
    return SDSP_OK;
}

int32_t sdsp_debug_set_key_cert(int32_t fixed_margins) {
    test_hooks().key_cert_fixed.store(fixed_margins != 0);
    return SDSP_OK;
}

int32_t sdsp_debug_mem_info(int32_t device, uint64_t* free_bytes, uint64_t* total_bytes) {
    try {
        SDSP_HIP_CHECK(hipSetDevice(device));
        size_t fr = 0, to = 0;
        SDSP_HIP_CHECK(hipMemGetInfo(&fr, &to));
        if (free_bytes) *free_bytes = fr;
        if (total_bytes) *total_bytes = to;
        return SDSP_OK;
    } catch (const std::exception&) {
        return SDSP_ERR_PROCESSING;
    }
}

// the PCI bus id of a HIP device ("0000:c1:00.0"): the benchmark reads that card's shader clock
// from sysfs (HIP device numbers are not the driver's card numbers under HIP_VISIBLE_DEVICES)
int32_t sdsp_debug_device_pci_bus_id(int32_t device, char* out, uint32_t len) {
    if (!out || len < 13) return SDSP_ERR_INVALID_INPUT;
    return hipDeviceGetPCIBusId(out, (int)len, device) == hipSuccess ? SDSP_OK : SDSP_ERR_PROCESSING;
}

// test probe: device allocations the engine has made so far (count, bytes)
int32_t sdsp_debug_alloc_stats(uint64_t* n_allocs, uint64_t* bytes) {
    if (n_allocs) *n_allocs = g_alloc_n.load();
    if (bytes) *bytes = g_alloc_bytes.load();
    return SDSP_OK;
}

int32_t sdsp_probe_stft(int32_t device, uint64_t nfft, uint64_t hop, uint64_t n_tracks, uint64_t len, int32_t reps,
                        int32_t stride, double* ms_per_launch, double* bytes_per_launch) {
    try {
        if (!stft_size_ok((int)std::min<uint64_t>(nfft, 1u << 30)) || len < nfft || hop == 0 || n_tracks == 0 || reps <= 0)
            return SDSP_ERR_INVALID_INPUT;
        DeviceCtx& c = device_ctx(device);
        std::lock_guard<std::mutex> lk(c.mu);
        SDSP_HIP_CHECK(hipSetDevice(device));
        const uint64_t F = (len - nfft) / hop + 1, total = F * n_tracks;
        const int bins = (int)nfft / 2 + 1;
        if (stride < bins) stride = (bins + 3) & ~3;
        FftTables& tb = c.tables((int)nfft, true);
        DevBuf x, pfx, off, g, row0, mags, fmax;
        x.ensure(n_tracks * len * 4);
        mags.ensure(total * (uint64_t)stride * 4);
        fmax.ensure(total * 4);
        std::vector<float> noise(len);
        uint32_t st = 12345u;
        for (auto& v : noise) {
            st = st * 1664525u + 1013904223u;
            v = ((float)(st >> 8) / 16777216.0f - 0.5f) * 0.6f;
        }
        SDSP_HIP_CHECK(hipMemcpy(x.p, noise.data(), len * 4, hipMemcpyHostToDevice));
        for (uint64_t t = 1; t < n_tracks; t++)
            SDSP_HIP_CHECK(hipMemcpy(x.as<float>() + t * len, x.p, len * 4, hipMemcpyDeviceToDevice));
        std::vector<uint64_t> pf(n_tracks + 1), o(n_tracks), r0(n_tracks);
        std::vector<float> gv(n_tracks, 0.8912509f);
        for (uint64_t t = 0; t <= n_tracks; t++) pf[t] = t * F;
        for (uint64_t t = 0; t < n_tracks; t++) {
            o[t] = t * len;
            r0[t] = t * F;
        }
        const bool frame_parallel = test_hooks().stft_frame_parallel.load() != 0;  // test hook
        const std::vector<uint64_t> sp = stft_strips(pf);
        DevBuf strips, redo;
        strips.ensure(sp.size() * 8);
        redo.ensure((total + 1) * 4);
        SDSP_HIP_CHECK(hipMemcpy(strips.p, sp.data(), sp.size() * 8, hipMemcpyHostToDevice));
        pfx.ensure(pf.size() * 8);
        off.ensure(o.size() * 8);
        row0.ensure(r0.size() * 8);
        g.ensure(gv.size() * 4);
        SDSP_HIP_CHECK(hipMemcpy(pfx.p, pf.data(), pf.size() * 8, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(off.p, o.data(), o.size() * 8, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(row0.p, r0.data(), r0.size() * 8, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(g.p, gv.data(), gv.size() * 4, hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        SDSP_HIP_CHECK(hipEventCreate(&e0));
        SDSP_HIP_CHECK(hipEventCreate(&e1));
        auto launch = [&]() {
            launch_stft((int)nfft, nfft != 8192, x.as<float>(), pfx.as<uint64_t>(), (int)n_tracks, total,
                        off.as<uint64_t>(), g.as<float>(), (int)hop, tb.window.as<float>(),
                        stft_twp(tb, (int)nfft, nfft != 8192), stft_rtp(tb, (int)nfft, nfft != 8192), mags.as<float>(), row0.as<uint64_t>(), stride, fmax.as<float>(), c.stream,
                        frame_parallel ? nullptr : strips.as<uint64_t>(), sp.back(), redo.as<uint32_t>());
        };
        launch();  // warm: first touch of the output pages
        SDSP_HIP_CHECK(hipEventRecord(e0, c.stream));
        for (int r = 0; r < reps; r++) launch();
        SDSP_HIP_CHECK(hipEventRecord(e1, c.stream));
        SDSP_HIP_CHECK(hipGetLastError());
        SDSP_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        SDSP_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        *ms_per_launch = ms / reps;
        *bytes_per_launch = (double)n_tracks * (4.0 * (double)len + 4.0 * (double)F * (double)bins);
        return SDSP_OK;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "sdsp_probe_stft: %s\n", e.what());
        return SDSP_ERR_PROCESSING;
    }
}

// Stage probe: STFT magnitudes of one host buffer (x*gain framed at hop), frames x (nfft/2+1).
int32_t sdsp_debug_stft(const float* host_x, uint64_t n, uint64_t nfft, uint64_t hop, float gain, float* host_out,
                        float* host_frame_max, int32_t device) {
    try {
        if (!stft_size_ok((int)std::min<uint64_t>(nfft, 1u << 30)) || n < nfft || hop == 0) return SDSP_ERR_INVALID_INPUT;
        DeviceCtx& c = device_ctx(device);
        std::lock_guard<std::mutex> lk(c.mu);
        SDSP_HIP_CHECK(hipSetDevice(device));
        const uint64_t frames = (n - nfft) / hop + 1;
        const int bins = (int)nfft / 2 + 1;
        const int stride = (bins + 3) & ~3;
        FftTables& tb = c.tables((int)nfft, true);
        DevBuf x, pfx, off, g, row0, mags, fmax;
        x.ensure(n * 4);
        mags.ensure(frames * stride * 4);
        fmax.ensure(frames * 4);
        pfx.ensure(16);
        off.ensure(8);
        g.ensure(4);
        row0.ensure(8);
        const uint64_t pf[2] = {0, frames}, o0 = 0, r0 = 0;
        const std::vector<uint64_t> sp = stft_strips(std::vector<uint64_t>{0, frames});
        DevBuf strips, redo;
        strips.ensure(16);
        redo.ensure((frames + 1) * 4);
        SDSP_HIP_CHECK(hipMemcpy(strips.p, sp.data(), 16, hipMemcpyHostToDevice));
        // test hook: the frame-parallel kernel (k_stft_mag) for every hop
        const bool frame_parallel = test_hooks().stft_frame_parallel.load() != 0;
        SDSP_HIP_CHECK(hipMemcpy(x.p, host_x, n * 4, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(pfx.p, pf, 16, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(off.p, &o0, 8, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(g.p, &gain, 4, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(row0.p, &r0, 8, hipMemcpyHostToDevice));
        launch_stft((int)nfft, nfft != 8192, x.as<float>(), pfx.as<uint64_t>(), 1, frames, off.as<uint64_t>(),
                    g.as<float>(), (int)hop, tb.window.as<float>(), stft_twp(tb, (int)nfft, nfft != 8192),
                    stft_rtp(tb, (int)nfft, nfft != 8192), mags.as<float>(),
                    row0.as<uint64_t>(), stride, fmax.as<float>(), c.stream, frame_parallel ? nullptr : strips.as<uint64_t>(),
                    sp.back(), redo.as<uint32_t>());
        SDSP_HIP_CHECK(hipGetLastError());
        SDSP_HIP_CHECK(hipStreamSynchronize(c.stream));
        SDSP_HIP_CHECK(hipMemcpy2D(host_out, (size_t)bins * 4, mags.p, (size_t)stride * 4, (size_t)bins * 4,
                                   frames, hipMemcpyDeviceToHost));
        if (host_frame_max && nfft != 8192)
            SDSP_HIP_CHECK(hipMemcpy(host_frame_max, fmax.p, frames * 4, hipMemcpyDeviceToHost));
        return SDSP_OK;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "sdsp_debug_stft: %s\n", e.what());
        return SDSP_ERR_PROCESSING;
    }
}

// Stage probe: frame RMS (k_frame_rms_run / k_frame_rms) of n_tracks host tracks packed in one
// buffer (track t = host_x[offs[t] .. offs[t] + lens[t])), frames of fs samples every hop, the
// silence-trimming framing (a track shorter than fs has one frame of its length).  Writes the
// frames of all tracks in order to host_out (sum of frame counts).  per_frame = 1 forces the
// per-frame kernel.
int32_t sdsp_debug_frame_rms(const float* host_x, uint64_t n_total, const uint64_t* offs, const uint64_t* lens,
                             const float* gains, uint64_t n_tracks, uint64_t fs, uint64_t hop, int32_t per_frame,
                             float* host_out, int32_t device) {
    try {
        if (n_tracks == 0 || fs == 0 || hop == 0 || fs > (1u << 20) || hop > (1u << 20)) return SDSP_ERR_INVALID_INPUT;
        for (uint64_t t = 0; t < n_tracks; t++)
            if (offs[t] + lens[t] > n_total) return SDSP_ERR_INVALID_INPUT;
        DeviceCtx& c = device_ctx(device);
        std::lock_guard<std::mutex> lk(c.mu);
        SDSP_HIP_CHECK(hipSetDevice(device));
        std::vector<uint64_t> pfx(n_tracks + 1, 0);
        for (uint64_t t = 0; t < n_tracks; t++) {
            const uint64_t n = lens[t];
            pfx[t + 1] = pfx[t] + (n >= fs ? (n - fs) / hop + 1 : (n > 0 ? 1 : 0));
        }
        const uint64_t total = pfx[n_tracks];
        DevBuf x, p, o, l, g, out;
        x.ensure(std::max<uint64_t>(n_total, 1) * 4);
        p.ensure(pfx.size() * 8);
        o.ensure(n_tracks * 8);
        l.ensure(n_tracks * 8);
        g.ensure(n_tracks * 4);
        out.ensure(std::max<uint64_t>(total, 1) * 4);
        if (n_total) SDSP_HIP_CHECK(hipMemcpy(x.p, host_x, n_total * 4, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(p.p, pfx.data(), pfx.size() * 8, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(o.p, offs, n_tracks * 8, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(l.p, lens, n_tracks * 8, hipMemcpyHostToDevice));
        SDSP_HIP_CHECK(hipMemcpy(g.p, gains, n_tracks * 4, hipMemcpyHostToDevice));
        launch_frame_rms(x.as<float>(), o.as<uint64_t>(), g.as<float>(), l.as<uint64_t>(), p.as<uint64_t>(),
                         (int)n_tracks, total, (int)fs, (int)hop, out.as<float>(), c.stream, per_frame != 0);
        SDSP_HIP_CHECK(hipGetLastError());
        SDSP_HIP_CHECK(hipStreamSynchronize(c.stream));
        if (total) SDSP_HIP_CHECK(hipMemcpy(host_out, out.p, total * 4, hipMemcpyDeviceToHost));
        return SDSP_OK;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "sdsp_debug_frame_rms: %s\n", e.what());
        return SDSP_ERR_PROCESSING;
    }
}

}  // extern "C"
