"""GPU STFT kernel vs the CPU restatement: bit-exact (same specified FFT arithmetic)."""
import numpy as np
import pytest

import oracle
import sdsp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("frame_parallel", [False, True])
@pytest.mark.parametrize("nfft,hop", [(2048, 512), (2048, 256), (2048, 1024), (8192, 512), (8192, 1024), (2048, 300),
                                      (8192, 256)])
def test_stft_bit_exact(nfft, hop, frame_parallel):
    """The sliding-strip kernel (hops k_stft_slide serves; strips of 64 frames, a partial last
    strip) and the frame-parallel kernel (every hop; the stft_frame_parallel test hook forces it)."""
    rng = np.random.default_rng(nfft + hop)
    x = (rng.standard_normal(44100 * 3) * 0.3).astype(np.float32)
    gain = np.float32(0.8912509)
    with sdsp.test_hooks(stft_frame_parallel=frame_parallel):
        got, fmax = sdsp.debug_stft(x, nfft, hop, gain)
    ref = oracle.stft((x * gain).astype(np.float32), nfft, hop)
    assert got.shape == ref.shape
    mism = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert mism == 0, f"{mism} of {ref.size} magnitudes differ (max abs diff {np.max(np.abs(got - ref))})"
    if nfft == 2048:
        assert np.array_equal(fmax, ref.max(axis=1))


@pytest.mark.parametrize("nfft,hop", [(64, 16), (128, 37), (256, 128), (512, 256), (1024, 512), (1024, 441),
                                      (4096, 512), (4096, 1000), (16384, 2048)])
def test_stft_general_sizes_bit_exact(nfft, hop):
    """k_stft_gen (frame sizes other than the tuned 2048 / 8192: AnalysisConfig::frame_size is a
    free power of two): radix-4 stages, the radix-2 stage when log2(N/2) is odd (64, 256, 1024,
    4096, 16384), odd hops (unaligned frames), 128 KB of LDS at N = 16384; bit-exact magnitudes and
    frame maxima."""
    rng = np.random.default_rng(nfft * 3 + hop)
    x = (rng.standard_normal(44100 * 2) * 0.3).astype(np.float32)
    x[20000:30000] = 0.0
    x[40000:45000] = (rng.standard_normal(5000) * 1e-30).astype(np.float32)
    gain = np.float32(0.8912509)
    got, fmax = sdsp.debug_stft(x, nfft, hop, gain)
    ref = oracle.stft((x * gain).astype(np.float32), nfft, hop)
    assert got.shape == ref.shape
    mism = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert mism == 0, f"{mism} of {ref.size} magnitudes differ (max abs diff {np.max(np.abs(got - ref))})"
    assert np.array_equal(fmax, ref.max(axis=1))


@pytest.mark.parametrize("nfft", [32, 3000, 32768])
def test_stft_sizes_refused(nfft):
    """Sizes outside the powers of two in [64, 16384] are refused with INVALID_INPUT."""
    x = np.zeros(70000, np.float32)
    with pytest.raises(sdsp.AnalysisError):
        sdsp.debug_stft(x, nfft, 512)


@pytest.mark.parametrize("nfft,hop", [(2048, 512), (8192, 512), (2048, 256)])
def test_stft_silence_and_subnormal_scale(nfft, hop):
    """Digital silence (|X|^2 = 0: the fast sqrt's zero case) and frames of ~1e-30-scale samples
    ((2^33 |X|)^2 below 2^-96, outside the fast sqrt's exact range: the sliding kernel lists those
    frames and k_stft_mag redoes them) next to ordinary frames, bit-exact."""
    rng = np.random.default_rng(nfft + 7 * hop)
    n = 44100 * 2
    x = (rng.standard_normal(n) * 0.3).astype(np.float32)
    x[10000:40000] = 0.0
    x[50000:70000] = (rng.standard_normal(20000) * 1e-30).astype(np.float32)
    got, fmax = sdsp.debug_stft(x, nfft, hop, np.float32(1.0))
    ref = oracle.stft(x, nfft, hop)
    mism = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert mism == 0, f"{mism} of {ref.size} magnitudes differ"
    p2 = (ref.astype(np.float64) * 2.0 ** 33) ** 2
    assert np.any(ref == 0.0) and np.any((p2 > 0) & (p2 < 2.0 ** -96))  # both special ranges are exercised


@pytest.mark.parametrize("frame_parallel", [False, True])
@pytest.mark.parametrize("nfft,hop", [(8192, 512), (8192, 1024), (2048, 512), (2048, 256)])
def test_stft_mostly_subnormal_scale_frames(nfft, hop, frame_parallel):
    """More than half of the frames (here ~90 %) have magnitudes of subnormal scale, so the sliding
    kernel lists most of the launch on its redo list: each frame is listed at most once (the 4
    waves of an 8192-point frame OR one flag), so the list never outgrows its capacity of one
    entry per frame; bit-exact against the restatement."""
    rng = np.random.default_rng(nfft + 11 * hop)
    n = 44100 * 4
    x = (rng.standard_normal(n) * 1e-30).astype(np.float32)
    x[: n // 12] = (rng.standard_normal(n // 12) * 0.3).astype(np.float32)
    with sdsp.test_hooks(stft_frame_parallel=frame_parallel):
        got, fmax = sdsp.debug_stft(x, nfft, hop, np.float32(1.0))
    ref = oracle.stft(x, nfft, hop)
    mism = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert mism == 0, f"{mism} of {ref.size} magnitudes differ"
    p2 = (ref.astype(np.float64) * 2.0 ** 33) ** 2
    tiny_frames = np.count_nonzero(np.any((p2 > 0) & (p2 < 2.0 ** -96), axis=1))
    assert tiny_frames > 0.5 * ref.shape[0], (tiny_frames, ref.shape[0])


@pytest.mark.parametrize("frame_parallel", [False, True])
@pytest.mark.parametrize("nfft,hop", [(8192, 512), (2048, 512), (2048, 300), (4096, 1000), (1024, 256)])
def test_stft_overflow_rule(nfft, hop, frame_parallel):
    """Unnormalised int-scale input (samples ~2^24, e.g. int24 / int32 PCM passed as float with
    enable_normalization = false): with the window's 2^32 the frame's |Y|^2 = 2^66 |X|^2
    overflows f32, where the reference's (re*re + im*im) does not (extractor.rs:352).  The spec's
    overflow rule re-evaluates those frames in the reference's range: bit-exact against the
    restatement, finite, and within 1e-5 (relative to the frame peak) of numpy's float64 FFT."""
    rng = np.random.default_rng(nfft + 13 * hop)
    n = 44100 * 2
    t = np.arange(n, dtype=np.float64)
    x = (np.sin(2 * np.pi * 441.0 * t / 44100) * 2.0 ** 24 + rng.standard_normal(n) * 2.0 ** 18).astype(np.float32)
    x[n // 2:] *= np.float32(1e-6)  # quiet half: ordinary frames beside the overflowing ones
    with sdsp.test_hooks(stft_frame_parallel=frame_parallel):
        got, fmax = sdsp.debug_stft(x, nfft, hop, np.float32(1.0))
    ref = oracle.stft(x, nfft, hop)
    mism = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert mism == 0, f"{mism} of {ref.size} magnitudes differ"
    assert np.all(np.isfinite(ref))
    assert np.any(ref.astype(np.float64) >= 2.0 ** 31)  # the rule is exercised
    w = np.float32(0.5) * (np.float32(1) - np.cos((np.float32(2 * np.pi) * np.arange(nfft, dtype=np.float32) /
                                                   np.float32(nfft - 1)).astype(np.float32)))
    for f in (0, ref.shape[0] // 4, ref.shape[0] - 1):
        fr = x[f * hop: f * hop + nfft].astype(np.float64) * w.astype(np.float64)
        m64 = np.abs(np.fft.rfft(fr))
        assert np.max(np.abs(ref[f] - m64)) <= 1e-5 * max(m64.max(), 1e-30), f
