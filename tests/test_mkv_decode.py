"""Matroska / WebM audio (stratum-dsp_amd/csrc/host_mkv.hip) through the C ABI
(sdsp_decode_audio_file), on the CPU.

The reference reads Matroska through symphonia's MKV reader (Cargo.toml:15, features = ["all"]).
The files here are written from the Matroska / EBML specification around streams of the test
encoders (tests/flac_enc.py, alac_enc.py, vorbis_enc.py) and raw PCM; each decode must equal the
same stream's decode from its native container (PCM, FLAC, ALAC: exactly; Vorbis: the encoder's
synthesis within float32 rounding).  Covered: SimpleBlocks without lacing and with Xiph, EBML
and fixed-size lacing, BlockGroups, an unknown-size Cluster, a video track ahead of the audio
one, little / big-endian integer and IEEE float PCM, and the named errors (MP3, AAC).  Parity
against symphonia itself is unpinned.
"""
import struct

import numpy as np
import pytest

import alac_enc as ae
import flac_enc as fe
import sdsp
import vorbis_enc as ve

F32 = np.float32


def _vint_size(n, width=None):
    width = width or next(w for w in range(1, 9) if n < (1 << (7 * w)) - 1)
    return bytes([((1 << (8 - width)) | (n >> (8 * (width - 1)))) & 0xFF]) + (n & ((1 << (8 * (width - 1))) - 1)).to_bytes(width - 1, "big")


def _el(eid, payload, unknown=False):
    idb = eid.to_bytes((eid.bit_length() + 7) // 8, "big")
    size = bytes([0x01, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF]) if unknown else _vint_size(len(payload))
    return idb + size + payload


def _uint(eid, v):
    return _el(eid, v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big"))


def _track(number, ttype, codec, rate=44100.0, channels=1, bits=None, priv=None):
    audio = _el(0xB5, struct.pack(">d", rate)) + _uint(0x9F, channels)
    if bits:
        audio += _uint(0x6264, bits)
    body = _uint(0xD7, number) + _uint(0x83, ttype) + _el(0x86, codec.encode())
    if priv is not None:
        body += _el(0x63A2, priv)
    if ttype == 2:
        body += _el(0xE1, audio)
    return _el(0xAE, body)


def _block(track, frames, lacing=None, simple=True):
    head = _vint_size(track, 1) + struct.pack(">h", 0)
    if lacing is None:
        assert len(frames) == 1
        body = head + bytes([0x80]) + frames[0]
    else:
        flag = {"xiph": 0x02, "fixed": 0x04, "ebml": 0x06}[lacing]
        body = head + bytes([0x80 | flag, len(frames) - 1])
        if lacing == "xiph":
            for f in frames[:-1]:
                n = len(f)
                while n >= 255:
                    body += b"\xff"
                    n -= 255
                body += bytes([n])
        elif lacing == "ebml":
            body += _vint_size(len(frames[0]))
            for a, b in zip(frames[:-2], frames[1:-1]):
                d = len(b) - len(a)
                w = next(w for w in range(1, 9) if abs(d) < (1 << (7 * w - 1)) - 1)
                body += _vint_size(d + (1 << (7 * w - 1)) - 1, w)
        body += b"".join(frames)
    if simple:
        return _el(0xA3, body)
    return _el(0xA0, _el(0xA1, body))


def _mkv(tracks, blocks, unknown_cluster=False):
    ebml = _el(0x1A45DFA3, _el(0x4282, b"matroska"))
    cluster = _el(0x1F43B675, _uint(0xE7, 0) + b"".join(blocks), unknown=unknown_cluster)
    seg = _el(0x1549A966, _uint(0x2AD7B1, 1000000)) + _el(0x1654AE6B, b"".join(tracks)) + cluster
    return ebml + _el(0x18538067, seg)


def _decode(tmp_path, data, name="t.mkv"):
    p = tmp_path / name
    p.write_bytes(data)
    return sdsp.decode_audio_file(str(p))


def _pcm(n, nch, seed):
    rng = np.random.default_rng(seed)
    return [np.clip(np.round(rng.standard_normal(n) * 6000), -32768, 32767).astype(np.int64) for _ in range(nch)]


@pytest.mark.parametrize("lacing", [None, "xiph", "ebml", "fixed"])
def test_mkv_pcm16_lacing(tmp_path, lacing):
    chans = _pcm(4096, 2, 1)
    raw = b"".join(struct.pack("<hh", int(a), int(b)) for a, b in zip(*chans))
    sizes = [1024, 2048, 1024, 3072, 1024, 1024, 4096, 1024, 1024, 512, 512] if lacing != "fixed" else [2048] * 8
    frames, o = [], 0
    for s in sizes:
        frames.append(raw[o:o + s])
        o += s
    assert o == len(raw)
    if lacing is None:
        blocks = [_block(2, [f], simple=(i % 2 == 0)) for i, f in enumerate(frames)]
    else:
        blocks = [_block(2, frames[:5], lacing), _block(2, frames[5:], lacing)]
    tracks = [_track(1, 1, "V_VP9"), _track(2, 2, "A_PCM/INT/LIT", 48000.0, 2, 16)]
    x, sr = _decode(tmp_path, _mkv(tracks, blocks, unknown_cluster=lacing == "xiph"))
    a, b = (c.astype(F32) / F32(32768.0) for c in chans)
    want = (((np.full(len(a), F32(-0.0)) + a).astype(F32) + b).astype(F32) / F32(2)).astype(F32)
    assert sr == 48000 and x.tobytes() == want.tobytes()


def test_mkv_pcm_big_and_float(tmp_path):
    v = _pcm(1000, 1, 2)[0] * 200
    raw = b"".join(int(s).to_bytes(3, "big", signed=True) for s in v)
    x, _ = _decode(tmp_path, _mkv([_track(1, 2, "A_PCM/INT/BIG", 44100.0, 1, 24)], [_block(1, [raw])]))
    assert x.tobytes() == (v.astype(F32) / F32(8388608.0)).tobytes()
    f = np.random.default_rng(3).uniform(-1, 1, 777)
    raw = b"".join(struct.pack("<d", s) for s in f)
    x, _ = _decode(tmp_path, _mkv([_track(1, 2, "A_PCM/FLOAT/IEEE", 44100.0, 1, 64)], [_block(1, [raw])]))
    assert x.tobytes() == f.astype(F32).tobytes()


def test_mkv_flac(tmp_path):
    bps = 16
    chans = [[c] for c in _pcm(1152, 1, 4)] + [[c] for c in _pcm(1152, 1, 5)]
    frames = [fe.frame(ch, bps, k) for k, ch in enumerate(chans)]
    native = fe.stream(frames, 44100, 1, bps)
    priv = bytearray(native[:4 + 38])
    priv[4] |= 0x80  # STREAMINFO as the last metadata block
    x, sr = _decode(tmp_path, _mkv([_track(1, 2, "A_FLAC", 44100.0, 1, priv=bytes(priv))],
                                   [_block(1, [f]) for f in frames]))
    assert sr == 44100 and x.tobytes() == fe.expected_mono(chans, bps).tobytes()


def test_mkv_alac(tmp_path):
    cfg = ae.Config(bit_depth=16, channels=2, frame_length=1024)
    chans = _pcm(2500, 2, 6)
    pk = [ae.frame(cfg, [c[s:s + 1024] for c in chans], [{"mix": (2, 1), "ch": [{"coefs": [500, -100], "den": 9}] * 2}])
          for s in range(0, 2500, 1024)]
    x, _ = _decode(tmp_path, _mkv([_track(1, 2, "A_ALAC", 44100.0, 2, priv=cfg.cookie())],
                                  [_block(1, pk[:2], "ebml"), _block(1, pk[2:])]))
    assert x.tobytes() == ae.expected_mono(cfg, chans).tobytes()


def test_mkv_vorbis(tmp_path):
    pattern = [1, 0, 0, 1, 1]
    bs = [256, 2048]
    span = sum(bs[pattern[k - 1]] // 4 + bs[pattern[k]] // 4 for k in range(1, len(pattern)))
    t = np.arange(span) / 44100
    pk, _, exp = ve.encode([0.3 * np.sin(2 * np.pi * 440 * t)], 44100, pattern, rtype=1)
    h = ve.headers(1, 44100, 1)
    priv = bytes([2, len(h[0]), len(h[1])]) + b"".join(h)
    x, sr = _decode(tmp_path, _mkv([_track(1, 2, "A_VORBIS", 44100.0, 1, priv=priv)], [_block(1, [p]) for p in pk]),
                    "t.webm")
    assert sr == 44100 and x.shape == exp[0].shape
    assert float(np.max(np.abs(x - exp[0]))) <= 2e-6


@pytest.mark.parametrize("codec,name", [("A_MPEG/L3", "MPEG audio"), ("A_AAC", "AAC")])
def test_mkv_named_errors(tmp_path, codec, name):
    with pytest.raises(sdsp.AnalysisError) as e:
        _decode(tmp_path, _mkv([_track(1, 2, codec)], [_block(1, [b"\x00" * 8])]))
    assert name in str(e.value) and e.value.kind == "DecodingError"
