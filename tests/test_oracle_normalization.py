"""The oracle's RMS / LUFS / peak normalization (normalization.rs) against the reference's own
unit tests for it (normalization.rs:549-739, restated as properties: the reference holds no
golden vectors for this module) and against an independent numpy restatement of the RMS and
K-weighted LUFS arithmetic.  CPU only."""
import math

import numpy as np
import pytest

import oracle

F = np.float32


def sine(n, amp, sr):
    """generate_test_signal (normalization.rs:553-562), f32."""
    t = np.arange(n, dtype=F) / F(sr)
    return (F(amp) * np.sin(F(2.0) * F(np.pi) * F(440.0) * t)).astype(F)


def test_peak_normalization():
    st, y = oracle.normalize(sine(44100, 0.5, 44100.0), 0)
    assert st == 0
    peak = np.abs(y).max()
    assert abs(peak - 10 ** (-1 / 20)) < 0.01 and peak <= 1.0


def test_rms_normalization():
    st, y = oracle.normalize(sine(44100, 0.3, 44100.0), 1)
    assert st == 0
    rms = math.sqrt(float(np.sum(y.astype(np.float64) ** 2)) / y.size)
    assert abs(rms - 10 ** ((-14.0 + 3.0 - 1.0) / 20)) < 0.1
    assert np.abs(y).max() <= 1.0


def test_lufs_normalization():
    x = sine(48000 * 2, 0.5, 48000.0)
    st, y = oracle.normalize(x, 2, 48000)
    assert st == 0
    assert not np.array_equal(x, y), "gain should be applied"
    assert np.abs(y).max() <= 1.0


def test_silent_and_quiet():
    z = np.zeros(44100, F)
    for m in (0, 1, 2):
        st, y = oracle.normalize(z, m)
        assert st == 0 and np.array_equal(y, z)
    st, _ = oracle.normalize(sine(44100, 1e-6, 44100.0), 0)
    assert st == 0


def test_empty_and_low_rate():
    for m in (0, 1, 2):
        st, msg = oracle.normalize(np.zeros(0, F), m)
        assert st == 1 and msg == "Empty audio samples"
    st, msg = oracle.normalize(sine(100, 0.5, 2.0), 2, 2)
    assert st == 1 and msg == "Sample rate too low for LUFS calculation"


def _pow10(e):
    return F(oracle.libm("pow", np.array([10.0], F), np.array([e], F))[0])


def test_rms_restatement_bit_exact():
    """Sequential f32 sum of squares (Iterator::sum), then the gain, clip-limited."""
    rng = np.random.default_rng(5)
    for amp in (0.05, 0.3, 0.9):
        x = (rng.standard_normal(30001) * amp).astype(F)
        x[17] = F(amp * 4)  # a peak that makes the clip limit bite for the louder cases
        ss = np.cumsum(x * x, dtype=F)[-1]
        rms = F(np.sqrt(F(ss / F(x.size))))
        target = _pow10(F(F(F(F(-14.0) + F(3.0)) - F(1.0)) / F(20.0)))
        g = F(target / rms)
        peak = np.abs(x).max()
        if F(peak * g) > F(1.0):
            g = F(F(1.0) / peak)
        st, y = oracle.normalize(x, 1)
        assert st == 0
        assert np.array_equal(y, (x * g).astype(F)), amp


def _lufs_numpy(x, sr):
    fsr = F(sr)
    w0 = F(F(F(F(2.0) * F(np.pi)) * F(1681.9745)) / fsr)
    cw, sw = F(np.cos(w0)), F(np.sin(w0))
    alpha = F(F(sw / F(2.0)) * F(np.sqrt(F(F(1.0) / F(0.707)))))
    a0 = F(F(1.0) + alpha)
    b0 = F(F(F(F(1.0) + cw) / F(2.0)) / a0)
    b1 = F(F(-(F(1.0) + cw)) / a0)
    b2 = b0
    a1 = F(F(F(-2.0) * cw) / a0)
    a2 = F(F(F(1.0) - alpha) / a0)
    x1 = x2 = F(0.0)
    y = np.empty_like(x)
    for i, s in enumerate(x):
        o = F(F(b0 * s) + x1)
        x1 = F(F(F(b1 * s) + x2) - F(a1 * o))
        x2 = F(F(b2 * s) - F(a2 * o))
        y[i] = o
    block = int(F(F(fsr * F(400.0)) / F(1000.0)))
    gate = _pow10(F(F(F(-70.0) + F(0.691)) / F(10.0)))
    ms = []
    for st in range(0, y.size, block):
        seg = y[st:st + block]
        ms.append(F(np.cumsum(seg * seg, dtype=F)[-1] / F(seg.size)))
    g = [m for m in ms if m > gate]
    mean = F(np.cumsum(np.array(g, F), dtype=F)[-1] / F(len(g)))
    return F(F(-0.691) + F(F(10.0) * F(math.log10(mean))))


@pytest.mark.parametrize("sr", [22050, 48000])
def test_lufs_restatement(sr):
    """The K-weighted, gated loudness and the gain it implies, against numpy (the sin/cos/log10
    of numpy may differ from the C library's by an ulp, hence the tolerance)."""
    rng = np.random.default_rng(sr)
    x = (np.sin(np.arange(sr * 2) * 0.05) * 0.2 + rng.standard_normal(sr * 2) * 0.01).astype(F)
    x[: sr // 2] *= F(1e-5)  # a block below the gate
    lufs = _lufs_numpy(x, sr)
    g = 10 ** ((-14.0 - float(lufs)) / 20)
    peak = float(np.abs(x).max())
    tpl = 10 ** (-1 / 20)
    if peak * g > tpl:
        g = tpl / peak
    st, y = oracle.normalize(x, 2, sr)
    assert st == 0
    got = float(y[np.argmax(np.abs(x))] / x[np.argmax(np.abs(x))])
    assert abs(got - g) <= 1e-5 * g
