"""Seeded synthetic tracks for CPU-side tests (SURVEY.md §8d recipe).

kick on every beat (60/120/180 Hz at 0.6/0.3/0.1, e^-10t, 100 ms — the reference's own fixture
generator, scripts/generate_fixtures.py:41-61), an off-beat noise hat (30 ms, e^-60t, 0.15), a
sustained tonic triad of the key and a diatonic 8th-note line (3 harmonics each), peak 0.9.
The throughput bench generates its tracks on the device instead (sdsp_generate_synthetic).
"""
import numpy as np

MAJOR = [0, 2, 4, 5, 7, 9, 11]
MINOR = [0, 2, 3, 5, 7, 8, 10]


def track_params(seed):
    rng = np.random.default_rng(0x5EED0000 + seed)
    bpm = 70.0 + 0.5 * int(rng.integers(0, 221))
    mode = int(rng.integers(0, 2))
    tonic = int(rng.integers(0, 12))
    return rng, bpm, mode, tonic


def make_track(seed, seconds=30.0, sr=44100, bpm=None, mode=None, tonic=None, silence_pad=0.0):
    rng, bpm0, mode0, tonic0 = track_params(seed)
    bpm = bpm0 if bpm is None else bpm
    mode = mode0 if mode is None else mode
    tonic = tonic0 if tonic is None else tonic
    n = int(seconds * sr)
    t = np.arange(n, dtype=np.float64) / sr
    x = np.zeros(n, np.float64)
    beat = 60.0 / bpm
    # kicks
    kl = int(0.1 * sr)
    kt = np.arange(kl) / sr
    kick = (np.sin(2 * np.pi * 60 * kt) * 0.6 + np.sin(2 * np.pi * 120 * kt) * 0.3 +
            np.sin(2 * np.pi * 180 * kt) * 0.1) * np.exp(-kt * 10)
    hl = int(0.03 * sr)
    ht = np.arange(hl) / sr
    henv = np.exp(-ht * 60) * 0.15
    b = 0.0
    while b < seconds:
        s = int(b * sr)
        e = min(s + kl, n)
        x[s:e] += kick[: e - s]
        hs = int((b + beat / 2) * sr)
        if hs < n:
            he = min(hs + hl, n)
            x[hs:he] += rng.standard_normal(he - hs) * henv[: he - hs]
        b += beat
    # harmony: tonic triad (sustained) + diatonic 8th-note line
    scale = MAJOR if mode == 0 else MINOR
    root = 48 + tonic  # MIDI C3 + tonic
    triad = [root, root + scale[2], root + scale[4]]

    def tone(midi, tt):
        f = 440.0 * 2 ** ((midi - 69) / 12.0)
        return sum(np.sin(2 * np.pi * f * h * tt) / h for h in (1, 2, 3))

    for m in triad:
        x += 0.2 / 3 * tone(m, t)
    step = beat / 2
    k = 0
    while k * step < seconds:
        s = int(k * step * sr)
        e = min(int((k + 1) * step * sr), n)
        deg = int(rng.integers(0, 7))
        midi = root + 12 + scale[deg]
        seg = t[s:e] - t[s]
        env = np.exp(-seg * 3.0)
        x[s:e] += 0.2 * tone(midi, t[s:e]) * env / 1.5
        k += 1
    x *= 0.9 / np.max(np.abs(x))
    x = x.astype(np.float32)
    if silence_pad > 0:
        z = np.zeros(int(silence_pad * sr), np.float32)
        x = np.concatenate([z, x, z])
    return x, bpm, mode, tonic


def chord_stab_track(bpm=72.0, seconds=20.0, hat_amp=0.04, stab_s=0.4, sr=44100, seed=0):
    """Harmonic C-major stabs (e^-4t, stab_s long) on every beat and quiet 20-ms noise hats
    (e^-150t) on every half beat.  The full mix's tempogram locks onto the stabs, so the base
    estimate lands in the low trap zone [55, 80]; the percussive component carries the hats at
    twice the rate.  At the defaults the percussive tempogram fallback (src/lib.rs:587-683) is
    *accepted* (tempogram_percussive_used = true, BPM ~143.8): the input that exercises that
    branch's "taken" outcome."""
    rng = np.random.default_rng(seed)
    n = int(sr * seconds)
    t = np.arange(n) / sr
    beat = 60.0 / bpm
    env = np.zeros(n)
    b = 0.0
    while b < seconds:
        i = int(b * sr)
        e = min(n, i + int(stab_s * sr))
        env[i:e] = np.maximum(env[i:e], np.exp(-np.arange(e - i) / sr * 4.0))
        b += beat
    x = env * sum(np.sin(2 * np.pi * f * t) for f in (261.63, 329.63, 392.0)) / 3
    b, hl = 0.0, int(0.02 * sr)
    while b < seconds:
        i = int(b * sr)
        e = min(n, i + hl)
        x[i:e] += hat_amp * rng.standard_normal(e - i) * np.exp(-np.arange(e - i) / sr * 150)
        b += beat / 2
    return (x * 0.9 / np.abs(x).max()).astype(np.float32)
