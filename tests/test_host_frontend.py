"""Host-side front-end functions of the library, on the CPU (no GPU needed: pure host code).

* sdsp_compute_confidence against the reference's own unit tests (confidence.rs:309-517) and,
  bit for bit, against the f32 restatement in oracle/host_restate.py on random results;
* sdsp_key_name against Key::name's doc examples (result.rs:21-30);
* sdsp_decode_audio_file on WAV files of every supported sample format / channel layout
  (written here), against the reference examples' conversion rules restated in numpy, on the
  reference's own fixtures (== the hound-based loader of the reference's integration tests),
  and on malformed / unsupported inputs (decoding errors).
"""
import ctypes as C
import os
import struct
import wave

import numpy as np
import pytest

import host_restate as hr
import parity
import sdsp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _res(bpm, bc, kc, kcl, gs, warnings=(), flags=()):
    return {"bpm": bpm, "bpm_confidence": bc, "key_confidence": kc, "key_clarity": kcl, "grid_stability": gs,
            "metadata": {"flags": list(flags), "confidence_warnings": list(warnings)}}


# ---- compute_confidence: the reference's tests ----
def test_confidence_all_good():
    c = sdsp.compute_confidence(_res(120.0, 0.9, 0.8, 0.7, 0.85))
    assert c["bpm_confidence"] == np.float32(0.9) and c["key_confidence"] == np.float32(0.8)
    assert c["grid_stability"] == np.float32(0.85)
    assert abs(c["overall_confidence"] - 0.855) < 0.01


def test_confidence_bpm_failed():
    c = sdsp.compute_confidence(_res(0.0, 0.0, 0.8, 0.7, 0.85))
    assert c["bpm_confidence"] == 0.0 and c["key_confidence"] == np.float32(0.8)
    assert abs(c["overall_confidence"] - 0.48) < 0.01


def test_confidence_key_failed():
    c = sdsp.compute_confidence(_res(120.0, 0.9, 0.0, 0.0, 0.85))
    assert c["key_confidence"] == 0.0
    assert abs(c["overall_confidence"] - 0.54) < 0.01


def test_confidence_all_failed():
    c = sdsp.compute_confidence(_res(0.0, 0.0, 0.0, 0.0, 0.0))
    assert c["overall_confidence"] == 0.0 and c["confidence_level"] == "Low"


def test_confidence_with_warnings():
    c = sdsp.compute_confidence(_res(120.0, 0.9, 0.8, 0.7, 0.85, ["BPM detection failed: insufficient onsets"]))
    assert 0.0 < c["bpm_confidence"] < 0.9


def test_confidence_clamping_and_levels():
    c = sdsp.compute_confidence(_res(120.0, 1.5, -0.5, 0.7, 2.0))
    assert c["bpm_confidence"] <= 1.0 and c["key_confidence"] >= 0.0 and c["grid_stability"] <= 1.0
    assert 0.0 <= c["overall_confidence"] <= 1.0
    assert sdsp.compute_confidence(_res(120.0, 0.9, 0.8, 0.7, 0.85))["confidence_level"] == "High"


def test_confidence_key_clarity_adjustment():
    hi = sdsp.compute_confidence(_res(120.0, 0.9, 0.8, 0.7, 0.85))
    lo = sdsp.compute_confidence(_res(120.0, 0.9, 0.8, 0.1, 0.85))
    assert lo["key_confidence"] < hi["key_confidence"]


def test_confidence_matches_restatement_bitwise():
    rng = np.random.default_rng(7)
    warn_pool = ["BPM detection failed: insufficient onsets or estimation error",
                 "Low key detection confidence: 0.12 (may indicate ambiguous or atonal music)",
                 "Low key clarity: 0.10 (track may be atonal or have weak tonality)",
                 "Low beat grid stability: 0.31 (may indicate tempo variation)"]
    for _ in range(3000):
        v = rng.uniform(-0.3, 1.3, 5).astype(np.float32)
        bpm = float(rng.choice([0.0, -1.0, 92.5, 128.0, 174.25]))
        warns = [w for w in warn_pool if rng.random() < 0.3]
        flags = ["WeakTonality"] if rng.random() < 0.3 else []
        got = sdsp.compute_confidence(_res(bpm, v[0], v[1], v[2], v[3], warns, flags))
        ref = hr.compute_confidence(bpm, v[0], v[1], v[2], v[3], flags, warns)
        for k in ("bpm_confidence", "key_confidence", "grid_stability", "overall_confidence"):
            assert np.float32(got[k]).tobytes() == np.float32(ref[k]).tobytes(), (k, got, ref)
        assert got["flags"] == ref["flags"]
        assert got["confidence_level"] == hr.confidence_level(np.float32(ref["overall_confidence"]))


def test_key_name():
    lib = sdsp.lib()
    buf = C.create_string_buffer(8)
    for mode, tonic, name in [(0, 0, "C"), (0, 6, "F#"), (1, 9, "Am"), (1, 1, "C#m"), (0, 23, "B")]:
        n = lib.sdsp_key_name(mode, tonic, buf, 8)
        assert buf.value.decode() == name and n == len(name)


# ---- decode front-end ----
def _write_wav(path, tag, channels, sr, bits, payload, extensible=False, extra_chunks=b""):
    block = channels * bits // 8
    if extensible:
        guid = struct.pack("<H", tag) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
        fmt = struct.pack("<HHIIHHHHI", 0xFFFE, channels, sr, sr * block, block, bits, 22, bits, 0) + guid
    else:
        fmt = struct.pack("<HHIIHH", tag, channels, sr, sr * block, block, bits)
    body = b"WAVE" + extra_chunks + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    body += b"data" + struct.pack("<I", len(payload)) + payload + (b"\x00" if len(payload) % 2 else b"")
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


CASES = [  # kind, tag, bits, numpy dtype of the raw samples
    ("u8", 1, 8, np.uint8), ("s16", 1, 16, np.int16), ("s24", 1, 24, None), ("s32", 1, 32, np.int32),
    ("f32", 3, 32, np.float32), ("f64", 3, 64, np.float64), ("alaw", 6, 8, np.uint8), ("ulaw", 7, 8, np.uint8),
]


@pytest.mark.parametrize("kind,tag,bits,dt", CASES)
@pytest.mark.parametrize("channels", [1, 2, 3])
@pytest.mark.parametrize("ext", [False, True])
def test_decode_formats(tmp_path, kind, tag, bits, dt, channels, ext):
    rng = np.random.default_rng(bits * 10 + channels)
    n = 1001
    if kind in ("u8", "alaw", "ulaw"):
        raw = rng.integers(0, 256, (n, channels)).astype(np.uint8)
        payload = raw.tobytes()
    elif kind == "s24":
        raw = rng.integers(-(1 << 23), 1 << 23, (n, channels)).astype(np.int64)
        raw[0, 0], raw[1, 0] = -(1 << 23), (1 << 23) - 1
        u = (raw & 0xFFFFFF).astype(np.uint32)
        payload = np.stack([u & 0xFF, (u >> 8) & 0xFF, (u >> 16) & 0xFF], -1).astype(np.uint8).tobytes()
    elif kind in ("f32", "f64"):
        raw = rng.uniform(-1.5, 1.5, (n, channels)).astype(dt)
        raw[0, 0] = -0.0
        payload = raw.tobytes()
    else:
        info = np.iinfo(dt)
        raw = rng.integers(info.min, info.max, (n, channels), endpoint=True).astype(dt)
        raw[0, 0], raw[1, 0] = info.min, info.max
        payload = raw.tobytes()
    p = tmp_path / "x.wav"
    _write_wav(p, tag, channels, 22050, bits, payload, extensible=ext,
               extra_chunks=b"LIST" + struct.pack("<I", 3) + b"abc\x00")
    x, sr = sdsp.decode_audio_file(str(p))
    assert sr == 22050 and x.dtype == np.float32 and x.shape == (n,)
    ref = hr.wav_mono(kind, raw)
    assert x.tobytes() == ref.tobytes()


@pytest.mark.parametrize("name", ["120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"])
def test_decode_reference_fixtures(name):
    x, sr = sdsp.decode_audio_file(os.path.join(GOLDEN, name))
    y, sr2 = parity.load_wav(os.path.join(GOLDEN, name))
    assert sr == sr2 and x.tobytes() == y.astype(np.float32).tobytes()


def test_decode_errors(tmp_path):
    bad = tmp_path / "bad.wav"
    bad.write_bytes(b"not a wav file at all")
    with pytest.raises(sdsp.AnalysisError) as e:
        sdsp.decode_audio_file(str(bad))
    assert e.value.code == 2 and "Decoding error" in str(e.value)
    with pytest.raises(sdsp.AnalysisError):
        sdsp.decode_audio_file(str(tmp_path / "missing.wav"))
    p = tmp_path / "pcm12.wav"
    _write_wav(p, 1, 1, 44100, 12, b"\x00" * 30)
    with pytest.raises(sdsp.AnalysisError) as e:
        sdsp.decode_audio_file(str(p))
    assert "bits" in str(e.value)
    p = tmp_path / "adpcm.wav"
    _write_wav(p, 2, 1, 44100, 4, b"\x00" * 30)
    with pytest.raises(sdsp.AnalysisError):
        sdsp.decode_audio_file(str(p))
    p = tmp_path / "nodata.wav"
    fmt = struct.pack("<HHIIHH", 1, 1, 44100, 88200, 2, 16)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    p.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)
    with pytest.raises(sdsp.AnalysisError):
        sdsp.decode_audio_file(str(p))


def test_decode_truncated_data_keeps_whole_frames(tmp_path):
    raw = np.arange(-50, 50, dtype=np.int16).reshape(50, 2)
    p = tmp_path / "t.wav"
    _write_wav(p, 1, 2, 44100, 16, raw.tobytes())
    b = p.read_bytes()
    p.write_bytes(b[:-7])  # cut inside the last frames
    x, _ = sdsp.decode_audio_file(str(p))
    assert x.size == (raw.nbytes - 7) // 4
    assert x.tobytes() == hr.wav_mono("s16", raw[: x.size]).tobytes()
