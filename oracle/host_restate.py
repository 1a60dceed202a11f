"""Pure-Python restatements of the host-side (non-GPU) pieces of the front-ends, for the tests.

TEST INFRASTRUCTURE: imported only by tests/ as the checker of the library's host functions
(sdsp_compute_confidence, sdsp_decode_audio_file), never by the product path.

- compute_confidence: src/analysis/confidence.rs:121-307, in f32 (numpy float32 scalars, one
  rounding per operation, the reference's operation order).
- wav_mono: the conversion the reference's examples apply to each symphonia buffer type
  (examples/analyze_file.rs:58-171): S16 / 32768, S24 / 8388608, S32 / 2147483648,
  (U8 - 128) / 128, F64 as f32, F32 as is; several channels summed in order from -0.0
  (Iterator::sum) and divided by the channel count.  G.711 A-law / mu-law expand to S16.
"""
import numpy as np

F = np.float32
FLAGS = ["MultimodalBpm", "WeakTonality", "TempoVariation", "OnsetDetectionAmbiguous"]


def _clamp(x, lo, hi):
    """f32::clamp (NaN passes through)."""
    x = F(x)
    if x < lo:
        return F(lo)
    if x > hi:
        return F(hi)
    return x


def compute_confidence(bpm, bpm_confidence, key_confidence, key_clarity, grid_stability, flags=(), warnings=()):
    """confidence.rs:121-307 -> dict (bpm_confidence, key_confidence, grid_stability,
    overall_confidence, flags)."""
    # compute_bpm_confidence :247-268
    if F(bpm) <= F(0.0):
        b = F(0.0)
    else:
        b = _clamp(bpm_confidence, 0.0, 1.0)
        if any("BPM" in w for w in warnings):
            b = F(b * F(0.7))
    # compute_key_confidence :276-307
    if F(key_confidence) <= F(0.0):
        k = F(0.0)
    else:
        base = _clamp(key_confidence, 0.0, 1.0)
        kc = F(key_clarity)
        clarity_adj = F(0.6) if kc < F(0.2) else F(0.85) if kc < F(0.5) else F(1.0)
        warn = any(("key" in w or "Key" in w or "tonality" in w) for w in warnings)
        warning_adj = F(0.7) if warn else F(1.0)
        k = F(F(base * clarity_adj) * warning_adj)
    g = _clamp(grid_stability, 0.0, 1.0)
    # :131-147
    if b > 0 and k > 0:
        overall = _clamp(F(F(F(b * F(0.4)) + F(k * F(0.3))) + F(g * F(0.3))), 0.0, 1.0)
    elif b > 0:
        overall = F(b * F(0.6))
    elif k > 0:
        overall = F(k * F(0.6))
    else:
        overall = F(0.0)
    fl = list(flags)
    if b < F(0.3):
        fl.append("MultimodalBpm")
    if k < F(0.2):
        fl.append("WeakTonality")
    if g < F(0.3):
        fl.append("TempoVariation")
    return {"bpm_confidence": b, "key_confidence": k, "grid_stability": g, "overall_confidence": overall,
            "flags": fl}


def confidence_level(overall):
    """AnalysisConfidence::confidence_level, confidence.rs:186-228."""
    return "High" if overall >= F(0.7) else "Low" if overall < F(0.5) else "Medium"


def alaw_to_s16(a):
    """ITU-T G.711 A-law expansion (the Sun reference implementation)."""
    a ^= 0x55
    t = (a & 0x0F) << 4
    seg = (a & 0x70) >> 4
    if seg == 0:
        t += 8
    elif seg == 1:
        t += 0x108
    else:
        t = (t + 0x108) << (seg - 1)
    return t if a & 0x80 else -t


def ulaw_to_s16(u):
    """ITU-T G.711 mu-law expansion (the Sun reference implementation)."""
    u = ~u & 0xFF
    t = ((u & 0x0F) << 3) + 0x84
    t <<= (u & 0x70) >> 4
    return (0x84 - t) if u & 0x80 else (t - 0x84)


def wav_mono(kind, frames):
    """frames: integer/float array [n, channels] of decoded samples of `kind`
    ('u8', 's16', 's24', 's32', 'f32', 'f64', 'alaw', 'ulaw' -- the latter two as raw bytes)."""
    if kind == "alaw":
        frames, kind = np.vectorize(alaw_to_s16)(frames.astype(np.int64)), "s16"
    elif kind == "ulaw":
        frames, kind = np.vectorize(ulaw_to_s16)(frames.astype(np.int64)), "s16"
    if kind == "u8":
        v = (frames.astype(F) - F(128.0)) / F(128.0)
    elif kind == "s16":
        v = frames.astype(F) / F(32768.0)
    elif kind == "s24":
        v = frames.astype(F) / F(8388608.0)
    elif kind == "s32":
        v = frames.astype(F) / F(2147483648.0)
    elif kind == "f64":
        v = frames.astype(F)
    else:
        v = frames.astype(F)
    v = v.astype(F)
    if v.shape[1] == 1:
        return v[:, 0].copy()
    s = np.full(v.shape[0], F(-0.0), dtype=F)
    for c in range(v.shape[1]):
        s = (s + v[:, c]).astype(F)
    return (s / F(v.shape[1])).astype(F)
