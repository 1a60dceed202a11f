"""The oracle's opt-in key chroma front-ends (oracle/o_chroma.cpp).  CPU only.

Pinned two ways:
  * the reference's own chroma unit tests (src/features/chroma/extractor.rs:1505-1624), restated on
    the oracle: A4 maps to pitch class 9, unit L2 norms, soft and hard mapping give equal lengths;
  * independent float64 numpy restatements of each function's arithmetic (extractor.rs:66-177
    tuning, :393-481 chroma, :529-680 whitened HPCP peaks, :701-985 log-frequency chroma,
    :830-935 beat-synchronous chroma, :1369-1501 the key HPSS median mask), which must agree to
    float32 rounding.  The reference has no
    unit test of these numbers, so beyond the restated formulas their values are "parity unpinned".
"""
import math

import numpy as np
import pytest

import oracle

SR = 44100


def _sine(freqs, seconds=2.0, sr=SR, amps=None):
    t = np.arange(int(sr * seconds), dtype=np.float64) / sr
    amps = amps or [1.0] * len(freqs)
    x = sum(a * np.sin(2 * np.pi * f * t) for f, a in zip(freqs, amps))
    return (x / max(1.0, np.max(np.abs(x)))).astype(np.float32)


# ---- libm additions (sin, atan2): correctly rounded to within 1 ulp of float64 ----
def test_libm_sin_atan2():
    rng = np.random.default_rng(3)
    x = rng.uniform(-np.pi, np.pi, 20000).astype(np.float32)
    got = oracle.libm("sin", x)
    ref = np.sin(x.astype(np.float64)).astype(np.float32)
    assert np.max(np.abs(got.view(np.int32) - ref.view(np.int32))) <= 1
    y = rng.normal(size=20000).astype(np.float32)
    z = rng.normal(size=20000).astype(np.float32)
    got = oracle.libm("atan2", y, z)
    ref = np.arctan2(y.astype(np.float64), z.astype(np.float64)).astype(np.float32)
    assert np.max(np.abs(got.view(np.int32) - ref.view(np.int32))) <= 1
    sp = np.array([0.0, -0.0, 0.0, -0.0, 1.0, -1.0, 0.0], np.float32)
    sx = np.array([1.0, 1.0, -1.0, -1.0, 0.0, 0.0, -0.0], np.float32)
    got = oracle.libm("atan2", sp, sx)
    ref = np.arctan2(sp.astype(np.float64), sx.astype(np.float64)).astype(np.float32)
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))


# ---- extractor.rs:1563-1578 test_frame_to_chroma ----
def test_frame_to_chroma_kat():
    mag = np.zeros((1, 1025), np.float32)
    mag[0, int(440.0 * 2048 / SR)] = 1.0
    ch, en = oracle.chroma("plain", mag, fft_size=2048, soft=False)
    assert ch.shape == (1, 12)
    n = float(np.sqrt(np.sum(ch[0].astype(np.float64) ** 2)))
    assert abs(n - 1.0) < 0.01 or n < 1e-10
    assert en[0] == 1.0


# ---- extractor.rs:1524-1561 test_extract_chroma_basic and :1596-1623 test_soft_chroma_mapping ----
@pytest.mark.parametrize("soft", [True, False])
def test_extract_chroma_a4(soft):
    spec = oracle.stft(_sine([440.0]), 2048, 512)
    ch, _ = oracle.chroma("plain", spec, fft_size=2048, soft=soft)
    assert ch.shape[0] == spec.shape[0] > 0
    norms = np.sqrt(np.sum(ch.astype(np.float64) ** 2, axis=1))
    assert np.all((np.abs(norms - 1.0) < 0.01) | (norms < 1e-10))
    assert ch[:, 9].mean() > 0.1
    assert int(np.argmax(ch.mean(axis=0))) == 9


# ---- numpy float64 restatements ----
def _semitone(f, tuning=0.0):
    return 12.0 * np.log2(f / 440.0) + 57.0 - tuning


def _soft(pc, s, contrib, sigma):
    spc = s % 12.0
    prim = int(round(spc)) % 12  # f32::round is half away from zero; spc >= 0
    for off in (-1, 0, 1):
        tc = (prim + off) % 12
        d = abs(spc - tc)
        d = min(d, 12.0 - d)
        pc[tc] += contrib * math.exp(-d * d / (2 * sigma * sigma))


def np_chroma(spec, sr, fft, soft, sigma, tuning):
    fres = sr / fft
    out = np.zeros((spec.shape[0], 12))
    for t, row in enumerate(spec.astype(np.float64)):
        pc = out[t]
        for b, m in enumerate(row):
            f = b * fres
            if f < 100.0:
                continue
            if f > min(5000.0, sr / 2) or f >= sr / 2:
                break
            s = _semitone(f, tuning)
            mag = max(m, 0.0) ** 0.6
            if soft:
                _soft(pc, s, mag, sigma)
            else:
                pc[int(math.floor(s + 0.5)) % 12] += mag
        n = np.sqrt(np.sum(pc * pc))
        if n > 1e-10:
            pc /= n
    return out


def np_tuning(spec, sr, fft, step, thr):
    fres = sr / fft
    ss = sc = sw = 0.0
    for t in range(0, spec.shape[0], step):
        row = spec[t].astype(np.float64)
        f = np.arange(row.size) * fres
        band = (f >= 80.0) & (f <= 2000.0)
        peak = row[band].max() if band.any() else 0.0
        if peak <= 1e-12:
            continue
        for b in np.nonzero(band & (row >= peak * thr))[0]:
            s = _semitone(f[b])
            r = s - math.floor(s + 0.5)
            w = math.sqrt(max(row[b], 0.0))
            ss += w * math.sin(2 * math.pi * r)
            sc += w * math.cos(2 * math.pi * r)
            sw += w
    if sw <= 1e-6 or math.hypot(ss, sc) / sw < 0.05:
        return 0.0
    return math.atan2(ss, sc) / (2 * math.pi)


def np_logfreq(spec, sr, fft):
    fres = sr / fft
    fmin, fmax = 100.0, min(5000.0, sr / 2 - 1.0)
    bmin = math.floor(_semitone(fmin))
    n = math.ceil(_semitone(fmax)) - bmin + 1
    out = np.zeros((spec.shape[0], 12))
    en = np.zeros(spec.shape[0])
    for t, row in enumerate(spec.astype(np.float64)):
        lf = np.zeros(n)
        for b, m in enumerate(row):
            f = b * fres
            if m <= 0 or f < fmin or f >= fmax:
                continue
            sf = _semitone(f) - bmin
            lo, hi = math.floor(sf), min(math.ceil(sf), n - 1)
            lf[lo] += m * (1.0 - (sf - lo))
            if hi != lo:
                lf[hi] += m * (sf - lo)
        for b in range(n):
            if lf[b] > 0:
                out[t, (bmin + b) % 12] += lf[b]
        nn = np.sqrt(np.sum(out[t] ** 2))
        if nn > 1e-10:
            out[t] /= nn
        en[t] = np.sum(lf * lf)
    return out, en


@pytest.fixture(scope="module")
def key_spec():
    x = _sine([261.63, 329.63, 392.0, 523.25, 110.0], seconds=3.0, amps=[1.0, 0.7, 0.8, 0.4, 0.6])
    rng = np.random.default_rng(5)
    x = x + (0.01 * rng.normal(size=x.size)).astype(np.float32)
    return oracle.stft(x, 8192, 512)


@pytest.mark.parametrize("soft,tuning", [(True, 0.0), (False, 0.0), (True, 0.07), (False, -0.04)])
def test_chroma_vs_numpy(key_spec, soft, tuning):
    spec = key_spec[::7]
    ch, en = oracle.chroma("plain", spec, soft=soft, tuning=tuning)
    ref = np_chroma(spec, SR, 8192, soft, 0.5, tuning)
    assert np.max(np.abs(ch - ref)) < 2e-4
    assert np.allclose(en, np.sum(spec.astype(np.float64) ** 2, axis=1), rtol=1e-4)


@pytest.mark.parametrize("detune", [0.0, 0.2, -0.3])
def test_tuning_vs_numpy(detune):
    f = [261.63 * 2 ** (detune / 12), 392.0 * 2 ** (detune / 12), 659.26 * 2 ** (detune / 12)]
    spec = oracle.stft(_sine(f, seconds=4.0), 8192, 512)
    got = oracle.tuning(spec, frame_step=5)
    ref = np_tuning(spec, SR, 8192, 5, 0.35)
    assert abs(got - ref) < 1e-4
    if detune != 0.0:
        assert np.sign(got) == np.sign(detune)


def test_logfreq_vs_numpy(key_spec):
    spec = key_spec[::5]
    ch, en = oracle.chroma("logfreq", spec)
    ref, ren = np_logfreq(spec, SR, 8192)
    assert np.max(np.abs(ch - ref)) < 1e-4
    assert np.allclose(en, ren, rtol=1e-4)
    # C major triad content: C, E, G dominate
    assert set(np.argsort(ch.mean(axis=0))[-3:]) == {0, 4, 7}


def test_beatsync(key_spec):
    spec = key_spec
    fd = np.float32(512) / np.float32(SR)
    beats = np.array([0.1, 0.6, 0.6, 1.2, 0.9, 2.5], np.float32)  # a duplicate and a reversed interval
    ch, en = oracle.chroma("beatsync", spec, beats=beats, tuning=0.03)
    fc, fe = oracle.chroma("plain", spec, tuning=0.03)
    assert ch.shape == (beats.size - 1, 12)
    ft = np.arange(spec.shape[0], dtype=np.float32) * fd
    for i in range(beats.size - 1):
        sel = (ft >= beats[i]) & (ft < beats[i + 1])
        if not sel.any():
            assert not ch[i].any() and en[i] == 0.0
            continue
        avg = fc[sel].astype(np.float64).mean(axis=0)
        avg /= np.sqrt(np.sum(avg * avg))
        assert np.max(np.abs(ch[i] - avg)) < 1e-5
        assert abs(en[i] - fe[sel].astype(np.float64).sum()) <= 1e-5 * fe[sel].sum()
    assert oracle.chroma("beatsync", spec, beats=beats[:1])[0].shape[0] == 0


def test_hpcp_tuning_shifts(key_spec):
    a, _ = oracle.chroma("hpcp", key_spec)
    b, _ = oracle.chroma("hpcp", key_spec, tuning=0.0)
    assert np.array_equal(a, b)
    c, _ = oracle.chroma("hpcp", key_spec, tuning=0.3)
    assert not np.array_equal(a, c)


def np_key_hpss(spec, sr, fft, step, tm, fm, p):
    F, B = spec.shape
    fres = np.float32(sr) / np.float32(fft)
    fmax = min(max(5000.0, 101.0), sr / 2)
    b0 = min(max(int(np.floor(np.float32(100.0) / fres)), 0), B)
    b1 = min(max(int(np.ceil(np.float32(fmax) / fres)), 0), B)
    san = np.where(np.isfinite(spec), np.maximum(spec, 0), 0).astype(np.float64)
    ds = san[::step, b0:b1]
    nds, nb = ds.shape
    h = np.zeros_like(ds)
    pe = np.zeros_like(ds)
    for t in range(nds):
        for b in range(nb):
            w = np.sort(ds[max(t - tm, 0):min(t + tm + 1, nds), b])
            h[t, b] = w[w.size // 2]
            w = np.sort(ds[t, max(b - fm, 0):min(b + fm + 1, nb)])
            pe[t, b] = w[w.size // 2]
    m = h ** p / (h ** p + pe ** p + 1e-12)
    out = np.zeros_like(san)
    k = np.minimum(np.arange(F) // step, nds - 1)
    out[:, b0:b1] = san[:, b0:b1] * m[k]
    return out


@pytest.mark.parametrize("step,tm,fm,p", [(4, 8, 8, 2.0), (1, 3, 5, 1.0), (3, 12, 2, 3.0)])
def test_key_hpss_vs_numpy(key_spec, step, tm, fm, p):
    spec = key_spec[:60]
    got = oracle.key_hpss(spec, step=step, time_margin=tm, freq_margin=fm, power=p)
    ref = np_key_hpss(spec, SR, 8192, step, tm, fm, p)
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-7 * float(np.max(spec)))
    assert not got[:, :18].any() and not got[:, 930:].any()  # outside [100, 5000] Hz -> 0
