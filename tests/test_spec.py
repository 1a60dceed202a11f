"""The arithmetic specification both engines implement (CPU only):

* include/sdsp_libm.h — f32 transcendentals, correctly rounded except within ~2^-51 of a
  rounding midpoint.  Checked against numpy's float64 functions rounded once to f32 (a
  float64 result can itself sit within its own error of an f32 midpoint, so a vanishing
  fraction of disagreements is tolerated).  powf(x, 2) == x*x exactly.
* include/sdsp_fft_spec.h — Stockham radix-4 FFT, real FFT and STFT magnitudes, checked
  against numpy's float64 FFT (the reference's rustfft is "parity unpinned", SURVEY §8c;
  float64 is the neutral yardstick): error <= 2e-6 * log2(N) of the frame's peak.
"""
import numpy as np
import pytest

import oracle

RNG = np.random.default_rng(1234)


def _f32_of(f64):
    return np.asarray(f64, dtype=np.float64).astype(np.float32)


def _mismatch_rate(got, want):
    return float(np.mean(got.view(np.uint32) != want.view(np.uint32)))


def test_ln_positive_range():
    x = np.concatenate([RNG.uniform(1.0, 2.0, 200000), np.exp(RNG.uniform(-80, 80, 200000)),
                        1.0 + RNG.uniform(0, 1e-4, 50000)]).astype(np.float32)
    assert _mismatch_rate(oracle.libm("ln", x), _f32_of(np.log(x.astype(np.float64)))) < 1e-5


def test_ln_known_hard_cases_are_pinned():
    # the 5 f32 inputs (of 2^31) where sd_logf is not correctly rounded (sdsp_libm.h)
    bits = np.array([0x3c413d3a, 0x41178feb, 0x4c5d65a5, 0x65d890d3, 0x6f31a8ec], np.uint32)
    x = bits.view(np.float32)
    got = oracle.libm("ln", x)
    want = _f32_of(np.log(x.astype(np.float64)))
    assert np.all(np.abs(got.astype(np.float64) - want.astype(np.float64)) <= np.spacing(np.abs(want)) * 1.01)


def test_ln_specials():
    x = np.array([0.0, -1.0, np.inf, 1.0, np.float32(1e-45)], np.float32)
    got = oracle.libm("ln", x)
    assert got[0] == -np.inf and np.isnan(got[1]) and got[2] == np.inf and got[3] == 0.0
    assert got[4] == np.float32(np.log(np.float64(x[4])))  # smallest subnormal


@pytest.mark.parametrize("op,fn,lo,hi", [("exp", np.exp, -80, 80), ("cos", np.cos, 0.0, 6.3),
                                         ("log10", np.log10, 1e-6, 1e6), ("log2", np.log2, 1e-6, 1e6)])
def test_transcendentals(op, fn, lo, hi):
    x = RNG.uniform(lo, hi, 300000).astype(np.float32)
    assert _mismatch_rate(oracle.libm(op, x), _f32_of(fn(x.astype(np.float64)))) < 1e-5


def test_pow():
    x = RNG.uniform(0.0, 4.0, 200000).astype(np.float32)
    assert np.array_equal(oracle.libm("pow", x, np.full_like(x, 2.0)), x * x)
    y = RNG.uniform(0.05, 1.0, x.size).astype(np.float32)
    want = _f32_of(np.power(x.astype(np.float64), y.astype(np.float64)))
    assert _mismatch_rate(oracle.libm("pow", x, y), want) < 1e-4


@pytest.mark.parametrize("M", [4, 8, 64, 512, 1024, 4096, 16384])
def test_fft_complex(M):
    z = (RNG.standard_normal(M) + 1j * RNG.standard_normal(M)).astype(np.complex64)
    got = oracle.fft(z)
    want = np.fft.fft(z.astype(np.complex128))
    assert np.max(np.abs(got - want)) <= 2e-6 * np.max(np.abs(want)) * np.log2(M)


@pytest.mark.parametrize("N", [2048, 8192])
def test_rfft(N):
    x = RNG.standard_normal(N).astype(np.float32)
    got = oracle.rfft(x)
    want = np.fft.rfft(x.astype(np.float64))
    assert np.max(np.abs(got - want)) <= 2e-6 * np.max(np.abs(want)) * np.log2(N)


@pytest.mark.parametrize("nfft,hop", [(2048, 512), (8192, 512), (2048, 256), (512, 128), (1024, 256), (4096, 1024),
                                      (16384, 4096)])
def test_stft_magnitudes(nfft, hop):
    """The STFT section of the spec (FMA complex products, no W^0 products, post-processing in
    FMA form; radix-2 last stage when log2(N/2) is odd)."""
    x = (0.5 * np.sin(2 * np.pi * 440.0 * np.arange(nfft * 4) / 44100.0) + 0.1 * RNG.standard_normal(nfft * 4))
    x = x.astype(np.float32)
    got = oracle.stft(x, nfft, hop)
    i = np.arange(nfft, dtype=np.float32)
    arg = (np.float32(2.0) * np.float32(np.pi) * i / np.float32(nfft - 1)).astype(np.float32)
    w = (np.float32(0.5) * (np.float32(1.0) - np.cos(arg.astype(np.float64)).astype(np.float32))).astype(np.float32)
    frames = (x.size - nfft) // hop + 1
    assert got.shape == (frames, nfft // 2 + 1)
    for f in range(frames):
        seg = (x[f * hop:f * hop + nfft] * w).astype(np.float64)
        want = np.abs(np.fft.rfft(seg))
        assert np.max(np.abs(got[f] - want)) <= 2e-6 * np.max(want) * np.log2(nfft)


def test_stft_silence_and_tiny_frames():
    """Digital silence gives exact zeros; frames of subnormal-scale samples stay finite and
    non-negative (the GPU's fast sqrt takes its general path there)."""
    n = 8192 * 3
    x = np.zeros(n, np.float32)
    x[8192:16384] = (RNG.standard_normal(8192) * 1e-38).astype(np.float32)
    for nfft in (2048, 8192):
        got = oracle.stft(x, nfft, 512)
        assert np.all(got[0] == 0.0) and np.all(np.isfinite(got)) and np.all(got >= 0.0)


def test_stft_short_input():
    assert oracle.stft(np.ones(100, np.float32), 2048, 512).shape == (0, 1025)


def test_logf_ge1_two_column_table_exhaustive(tmp_path):
    """k_features' ln(1 + max(X, 0)): sd_logf_ge1_t2 (the reduction k * (1/c) 2^-k without
    forming m or c) is bit-identical to sd_logf_ge1 on every f32 >= 1, +inf and NaN, and the
    branch-free sd_ln1p_max0_t2(v) to sd_logf_ge1_t2(1 + sd_maxf(v, 0)) on all 2^32 v, and
    the 9-bit-table, degree-4 sd_ln1p_x_t9_finite that k_features evaluates (round 5) to
    sd_logf_ge1 on every finite f32 >= 1 (tools/check_logf_ge1.c: ~6.4e9 inputs, ~10 s on 8
    threads)."""
    import shutil
    import subprocess
    from pathlib import Path
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "check_logf_ge1"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-march=x86-64-v3", "-fopenmp",
                    str(root / "tools" / "check_logf_ge1.c"), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.count(" 0 differ") == 3, out.stdout


def test_sqrt_is_powf_half_exhaustive(tmp_path):
    """HPCP's peak weights at the default power 0.5 take the correctly rounded sqrt where
    sd_sqrt_is_powf_half admits it (round 6); on every non-negative f32 the admitted sqrt equals
    sd_powf(x, 0.5f) bit for bit (tools/check_powf_half.c: 2.1e9 inputs, ~15 s on 8 threads).
    sqrtf alone would differ on 48 inputs, all within 2^-20 of a rounding midpoint."""
    import shutil
    import subprocess
    from pathlib import Path
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "check_powf_half"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-march=x86-64-v3", "-fopenmp",
                    str(root / "tools" / "check_powf_half.c"), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert " 0 differ" in out.stdout and "would differ on 48" in out.stdout, out.stdout
