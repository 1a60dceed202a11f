"""GPU STFT kernel vs the CPU restatement: bit-exact (same specified FFT arithmetic)."""
import numpy as np
import pytest

import oracle
import sdsp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("frame_parallel", [False, True])
@pytest.mark.parametrize("nfft,hop", [(2048, 512), (2048, 256), (2048, 1024), (8192, 512), (8192, 1024), (2048, 300),
                                      (8192, 256)])
def test_stft_bit_exact(nfft, hop, frame_parallel, monkeypatch):
    """The sliding-strip kernel (hops k_stft_slide serves; strips of 64 frames, a partial last
    strip) and the frame-parallel kernel (every hop; SDSP_STFT_FRAME_PARALLEL=1 forces it)."""
    if frame_parallel:
        monkeypatch.setenv("SDSP_STFT_FRAME_PARALLEL", "1")
    else:
        monkeypatch.delenv("SDSP_STFT_FRAME_PARALLEL", raising=False)
    rng = np.random.default_rng(nfft + hop)
    x = (rng.standard_normal(44100 * 3) * 0.3).astype(np.float32)
    gain = np.float32(0.8912509)
    got, fmax = sdsp.debug_stft(x, nfft, hop, gain)
    ref = oracle.stft((x * gain).astype(np.float32), nfft, hop)
    assert got.shape == ref.shape
    mism = np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert mism == 0, f"{mism} of {ref.size} magnitudes differ (max abs diff {np.max(np.abs(got - ref))})"
    if nfft == 2048:
        assert np.array_equal(fmax, ref.max(axis=1))


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
