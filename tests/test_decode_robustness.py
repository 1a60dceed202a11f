"""The decode front-end on damaged input (CPU): truncations and byte corruptions of valid files
of every supported container must either decode or fail with a decoding error -- never crash,
hang or read out of bounds (the examples skip packets that fail to decode, so damaged files
often still decode).  Seeded, a few hundred variants per format."""
import struct

import numpy as np
import pytest

import alac_enc as ae
import flac_enc as fe
import sdsp
import vorbis_enc as ve
import test_formats_decode as tf
import test_mkv_decode as tm


def _files():
    rng = np.random.default_rng(0)
    s16 = [np.clip(np.round(rng.standard_normal(3000) * 5000), -32768, 32767).astype(np.int64) for _ in range(2)]
    out = {}
    out["wav"] = tf._wav(1, 2, 44100, 4, 16, b"".join(struct.pack("<hh", int(a), int(b)) for a, b in zip(*s16)))
    out["aiff"] = tf._aiff(2, 16, 44100, 3000, tf._int_bytes(s16, 16, True))
    out["caf"] = tf._caf(44100, b"lpcm", 0, 4, 1, 2, 16, tf._int_bytes(s16, 16, True))
    frames = [fe.frame([c[k * 1000:(k + 1) * 1000] for c in s16], 16, k, assign="mid_side") for k in range(3)]
    out["flac"] = fe.stream(frames, 44100, 2, 16)
    out["ogg_flac"] = tf._ogg_pages(tf._flac_ogg_packets([[c[k * 1000:(k + 1) * 1000] for c in s16] for k in range(3)],
                                                         16, 44100, 2))
    cfg = ae.Config(bit_depth=16, channels=2, frame_length=1024)
    pk = [ae.frame(cfg, [c[s:s + 1024] for c in s16], [{"mix": (2, 1), "ch": [{"coefs": [400, -90], "den": 9}] * 2}])
          for s in range(0, 3000, 1024)]
    out["caf_alac"] = ae.caf(cfg, pk, 3000)
    out["m4a"] = ae.mp4(cfg, pk, [2, 1])
    pattern = [1, 0, 0, 1]
    vp, vg, _ = ve.encode([s16[0] / 40000.0, s16[1][:len(s16[0])] / 40000.0], 44100, pattern, rtype=2)
    out["vorbis"] = ve.ogg_stream(ve.headers(2, 44100, 2), vp, vg)
    out["mkv"] = tm._mkv([tm._track(1, 2, "A_ALAC", 44100.0, 2, priv=cfg.cookie())], [tm._block(1, pk[:2], "xiph"),
                                                                                    tm._block(1, pk[2:])])
    return out


FILES = _files()


@pytest.mark.parametrize("fmt", sorted(FILES))
def test_damaged_inputs_never_crash(tmp_path, fmt):
    data = FILES[fmt]
    x, _ = sdsp.decode_audio_file(str(_write(tmp_path, data)))  # the intact file decodes
    assert len(x) > 0
    rng = np.random.default_rng(hash(fmt) % (1 << 32))
    for trial in range(160):
        buf = bytearray(data)
        if trial % 4 == 0:
            buf = buf[:int(rng.integers(0, len(buf)))]
        else:
            for _ in range(int(rng.integers(1, 12))):
                buf[int(rng.integers(0, len(buf)))] = int(rng.integers(0, 256))
        try:
            y, sr = sdsp.decode_audio_file(str(_write(tmp_path, bytes(buf))))
            assert y.dtype == np.float32 and sr > 0
        except sdsp.AnalysisError as e:
            assert e.kind == "DecodingError", (fmt, trial, e.kind, str(e))


def _write(tmp_path, data):
    p = tmp_path / "f.bin"
    p.write_bytes(data)
    return p
