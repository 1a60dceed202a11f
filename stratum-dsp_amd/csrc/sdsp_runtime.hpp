// sdsp_runtime.hpp — host-side runtime internals (device contexts, buffers, launchers).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/stratum_hip.h"
#include "sdsp_device.hpp"

#define SDSP_HIP_CHECK(expr)                                                                              \
    do {                                                                                                  \
        hipError_t _e = (expr);                                                                           \
        if (_e != hipSuccess)                                                                             \
            throw sdsp::HipError(std::string(#expr) + " failed: " + hipGetErrorString(_e) + " at " __FILE__); \
    } while (0)

namespace sdsp {

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// Device allocations made by the engine (buffers and staging slots): count and bytes, for the
// tests' "a repeated call allocates nothing" check (sdsp_debug_alloc_stats).
void note_alloc(size_t bytes);

// Grow-only device allocation.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    // the engine streams that may still read the buffer (DeviceCtx::buf sets them); the caller's
    // own streams are never waited on here
    const std::vector<hipStream_t>* readers = nullptr;
    void ensure(size_t n) {
        if (n <= bytes) return;
        if (p) {
            // work queued on the engine's streams may still read the old buffer.  A buffer without
            // readers belongs to one synchronous probe call and is sized once; growing it again
            // would need a device-wide wait, which the engine never does
            if (!readers) throw HipError("DevBuf: an unowned buffer cannot grow");
            for (hipStream_t s : *readers) SDSP_HIP_CHECK(hipStreamSynchronize(s));
            SDSP_HIP_CHECK(hipFree(p));
        }
        p = nullptr;
        bytes = 0;
        const size_t want = n + n / 8 + 4096;
        SDSP_HIP_CHECK(hipMalloc(&p, want));
        note_alloc(want);
        bytes = want;
    }
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Per-size FFT tables (sdsp_fft_spec.h) + STFT windows, uploaded once per device.
struct FftTables {
    DevBuf tw;      // M-point complex twiddles (M = N/2)
    DevBuf rt;      // N/2+1 real-FFT post twiddles
    DevBuf window;  // N-point symmetric Hann (STFT sizes only)
    DevBuf stft_tw; // STFT sizes: the same twiddle values re-laid out per thread (k_stft.hip)
    DevBuf stft_rt; // STFT sizes: post twiddles in the kernel's pair order + specials
};

struct StageTimer;

struct DeviceCtx {
    int device = 0;
    hipStream_t stream = nullptr;   // main (tempo / beat) stream
    hipStream_t stream2 = nullptr;  // key-path stream, forked from and joined to `stream`
    hipStream_t stream3 = nullptr;  // key vote (k_key_vote), forked from stream2 after the chroma
    hipEvent_t vote_done = nullptr;  // the last key vote's end: the next chroma producer waits on it
    std::vector<hipStream_t> own;   // the streams above
    std::mutex mu;
    std::map<int, std::unique_ptr<FftTables>> fft;  // keyed by real FFT size N
    std::map<std::string, std::unique_ptr<DevBuf>> bufs;
    sdsp_stage_times last{};
    std::vector<uint8_t> last_near;  // per track of the last call: its key vote was near a decision (rerun)
    DevBuf& buf(const std::string& name) {
        auto& b = bufs[name];
        if (!b) {
            b.reset(new DevBuf());
            b->readers = &own;
        }
        return *b;
    }
    FftTables& tables(int N, bool with_window);
};

DeviceCtx& device_ctx(int device);

// Test hooks, set only through sdsp_debug_set_test_hooks / sdsp_debug_set_schedule (never from
// the environment): an injected chunk failure, a worker device list for sdsp_analyze_batch, the
// frame-parallel STFT kernel forced for every hop, and the schedule knobs below.
struct TestHooks {
    std::atomic<long> fail_chunk{-1};
    std::atomic<int> stft_frame_parallel{0};
    // schedule knobs (sdsp_debug_set_schedule; 0 = the product's schedule): the key path on the
    // main stream (per-kernel profiling), the key join at the end of each sub-batch, the
    // escalation passes without hop-512 row reuse, a per-stage host trace on stderr, the
    // sdsp_analyze_batch chunk size, and the sub-batch HBM budget in GB
    std::atomic<int> serial_streams{0}, no_key_defer{0}, no_row_reuse{0}, host_trace{0};
    std::atomic<uint64_t> batch_chunk_tracks{0};
    // sdsp_debug_set_key_cert: 1 = the key vote's fixed round-5 near-decision margins alone
    std::atomic<int> key_cert_fixed{0};
    std::atomic<double> hbm_budget_gb{0.0};
    std::mutex mu;
    std::vector<int> devices;
};
TestHooks& test_hooks();
std::vector<int> test_hooks_devices();

// STFT sizes with the tuned kernels (k_stft_mag / k_stft_slide: N = 2048, 8192).  Other powers of
// two in [STFT_GEN_MIN, STFT_GEN_MAX], and N = 8192 with frame maxima, run the general kernel
// k_stft_gen, which reads the spec's plain tables (FftTables::tw / rt); stft_twp / stft_rtp pick
// the tables launch_stft expects.
constexpr int STFT_GEN_MIN = 64, STFT_GEN_MAX = 16384;
bool stft_tuned(int N);
bool stft_size_ok(int N);
inline bool stft_general(int N, bool frame_max) { return !stft_tuned(N) || (N == 8192 && frame_max); }
inline const cx* stft_twp(FftTables& t, int N, bool frame_max) {
    return stft_general(N, frame_max) ? t.tw.as<cx>() : t.stft_tw.as<cx>();
}
inline const cx* stft_rtp(FftTables& t, int N, bool frame_max) {
    return stft_general(N, frame_max) ? t.rt.as<cx>() : t.stft_rt.as<cx>();
}

// Per-thread STFT twiddle tables (k_stft.hip), built from the sdsp_fft_spec.h tables (tw: N/2
// complex, rt: N/2+1 complex, interleaved) so every value is bit-identical to the spec's.
void stft_tables(int N, const std::vector<float>& tw, const std::vector<float>& rt, std::vector<float>* twp,
                 std::vector<float>* rtp);

// ---- kernel launchers (defined next to their kernels) ----
void launch_stft(int nfft, bool frame_max, const float* samples, const uint64_t* frame_pfx, int n_tracks,
                 uint64_t total_frames, const uint64_t* src_off, const float* gain, int hop, const float* window,
                 const cx* tw, const cx* rt, float* mags, const uint64_t* mag_row0, int stride, float* fmax,
                 hipStream_t st, const uint64_t* strip_pfx = nullptr, uint64_t n_strips = 0, uint32_t* redo = nullptr);
// the sliding-strip STFT (k_stft.hip): strip prefix over tracks from the frame prefix, and the
// (nfft, hop) pairs it serves
std::vector<uint64_t> stft_strips(const std::vector<uint64_t>& frame_pfx);
bool stft_slide_ok(int nfft, int hop);

}  // namespace sdsp
