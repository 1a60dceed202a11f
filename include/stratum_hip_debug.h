/*
 * stratum_hip_debug.h -- test and probe entry points of libstratum_hip.so.
 *
 * Not part of the drop-in boundary (include/stratum_hip.h): no reference interface corresponds to
 * these.  They exist for the parity tests (stage probes compared against the oracle), the
 * benchmark's isolated kernel timing and the failure-path tests.  The library reads no test switch
 * from the environment; the hooks below are set only through sdsp_debug_set_test_hooks.
 */
#ifndef STRATUM_HIP_DEBUG_H
#define STRATUM_HIP_DEBUG_H

#include <stdint.h>

#include "stratum_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Test hooks, process-wide: fail_chunk >= 0 makes sdsp_analyze_batch's chunk of that index throw
 * (the per-chunk failure path); devices[0..n_devices) replaces the device mask's worker list
 * (repeats allowed: two workers on device 0 run the multi-device chunk path on one GPU);
 * stft_frame_parallel != 0 forces the frame-parallel STFT kernel for every hop.  Reset with
 * (-1, NULL, 0, 0).
 */
int32_t sdsp_debug_set_test_hooks(int64_t fail_chunk, const int32_t* devices, uint32_t n_devices,
                                  int32_t stft_frame_parallel);

/*
 * Schedule knobs, process-wide (0 = the product's schedule): serial_streams != 0 runs the key path
 * on the main stream (per-kernel profiling); no_key_defer != 0 joins each sub-batch's key stream at
 * its own end instead of one sub-batch late; no_row_reuse != 0 recomputes the escalation passes'
 * hop-512 rows instead of reading the base pass's; host_trace != 0 prints per-stage host times on
 * stderr; batch_chunk_tracks > 0 sets sdsp_analyze_batch's chunk size (default 512 tracks);
 * hbm_budget_gb > 0 sets the sub-batch HBM budget (default: 80 % of free HBM / 1.125).  Every
 * setting gives the same results; the tests use them to reach the other schedules and the tools
 * to profile.  The Python layer maps SDSP_SERIAL_STREAMS, SDSP_NO_KEY_DEFER, SDSP_NO_ROW_REUSE,
 * SDSP_HOST_TRACE, SDSP_BATCH_CHUNK_TRACKS and SDSP_HBM_BUDGET_GB onto this call; the library
 * itself reads no environment variable.
 */
int32_t sdsp_debug_set_schedule(int32_t serial_streams, int32_t no_key_defer, int32_t no_row_reuse, int32_t host_trace,
                                uint64_t batch_chunk_tracks, double hbm_budget_gb);

/*
 * 1 when `cfg` at `sample_rate` takes the default key path's band-limited mask with HPCP frame
 * energies folded in 64-bin blocks (k_mask_rp / k_hpcp_band: key_confidence and key_clarity are
 * then a re-associated sum of the reference's), 0 when it keeps the reference's
 * single sequential energy fold, -1 on a NULL config or a zero rate.  No device is touched.
 */
int32_t sdsp_debug_key_energy_blocked(const sdsp_config* cfg, uint32_t sample_rate);

/*
 * Per track of the last analysis call on `device` (n entries): non-zero where the block-folded
 * key energies left a key decision within its margin, so the track's key path ran again with the
 * sequential energy fold (sdsp_stage_times.key_reruns counts them), else 0.  Bits: 1 a segment's
 * (or the slice's) within-mode argmax, 2 a segment clarity gate, 4 the final key gap, 8 the
 * weight-sum fallback, 16 a weight, energy or mode top outside the certificate's range (underflow,
 * no usable bound, near the 1e-9 normalisation guard).
 */
int32_t sdsp_debug_last_key_near(int32_t device, uint8_t* out, uint64_t n);

/*
 * The key vote's near-decision certificate on the default key path: 0 (default) the
 * rigorous bounds (per-frame energy bounds carried through the weights, raw scores, clarities and
 * the vote, with the fixed margins as floors); non-zero the fixed round-5 margins alone (A/B of the
 * flagged sets).  Process-wide; applies to the next analysis calls.
 */
int32_t sdsp_debug_set_key_cert(int32_t fixed_margins);

/* Free and total HBM bytes of `device` (the benchmark sizes its kernel probe by them). */
int32_t sdsp_debug_mem_info(int32_t device, uint64_t* free_bytes, uint64_t* total_bytes);

/* PCI bus id of HIP device `device` ("dddd:bb:dd.f", NUL-terminated; len >= 13). */
int32_t sdsp_debug_device_pci_bus_id(int32_t device, char* out, uint32_t len);

/* Device allocations the engine has made so far (count, bytes): "a repeated call allocates nothing". */
int32_t sdsp_debug_alloc_stats(uint64_t* n_allocs, uint64_t* bytes);

/*
 * STFT magnitudes of one host buffer (x * gain framed at hop), frames x (nfft/2 + 1) into host_out;
 * frame maxima into host_frame_max (NULL allowed; not for nfft 8192).
 */
int32_t sdsp_debug_stft(const float* host_x, uint64_t n, uint64_t nfft, uint64_t hop, float gain, float* host_out,
                        float* host_frame_max, int32_t device);

/*
 * Frame RMS of n_tracks host tracks (track t = host_x[offs[t] .. offs[t] + lens[t])), frames of fs
 * samples every hop, the silence-trimming framing; per_frame = 1 forces the per-frame kernel.
 */
int32_t sdsp_debug_frame_rms(const float* host_x, uint64_t n_total, const uint64_t* offs, const uint64_t* lens,
                             const float* gains, uint64_t n_tracks, uint64_t fs, uint64_t hop, int32_t per_frame,
                             float* host_out, int32_t device);

/*
 * Isolated STFT kernel timing: `reps` launches over n_tracks device-resident noise tracks of len
 * samples; mean launch time (HIP events on the launch stream) and algorithmic bytes per launch
 * (4 N_in + 4 F (nfft/2 + 1) per track).  stride 0 = the pipeline's row stride.
 */
int32_t sdsp_probe_stft(int32_t device, uint64_t nfft, uint64_t hop, uint64_t n_tracks, uint64_t len, int32_t reps,
                        int32_t stride, double* ms_per_launch, double* bytes_per_launch);

#ifdef __cplusplus
}
#endif

#endif /* STRATUM_HIP_DEBUG_H */
