"""Apple Lossless (stratum-dsp_amd/csrc/host_alac.hip) in CAF and ISO MP4 through the C ABI
(sdsp_decode_audio_file), on the CPU.

The reference decodes ALAC through symphonia (Cargo.toml:15, features = ["all"]); the streams here
are written by tests/alac_enc.py from Apple's published format, and ALAC is lossless, so the
decoded samples must be the encoded PCM exactly, through the examples' conversion
(examples/analyze_file.rs:25-180).  Parity against symphonia itself is unpinned.  Covered: the
adaptive Golomb coder (small and large values, escapes, zero runs), prediction with numactive 0,
31 and 4-16 coefficients, modes 0 and 15, stereo with and without mixing, "bytes shifted" low
bits at 24 and 32 bits, 20-bit samples, raw (escaped) elements, a partial last frame, both
containers (CAF with and without the 'frma' cookie wrapper; MP4 with several chunk runs), a
damaged packet (skipped, as the examples skip a packet that fails to decode) and the AAC error.
"""
import numpy as np
import pytest

import alac_enc as ae
import sdsp


def _sig(n, bits, seed, amp=0.5, noise=0.05, silence=()):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = amp * np.sin(2 * np.pi * t * (180 + 23 * seed) / 44100) + noise * rng.standard_normal(n)
    top = (1 << (bits - 1)) - 1
    v = np.clip(np.round(x * top), -top - 1, top).astype(np.int64)
    for a, b in silence:
        v[a:b] = 0
    return v


def _decode(tmp_path, data, name):
    p = tmp_path / name
    p.write_bytes(data)
    return sdsp.decode_audio_file(str(p))


def _frames(cfg, chans, specs):
    """Split channel arrays into frame_length packets, one spec per packet (cycled)."""
    n = len(chans[0])
    pk = []
    for k, s in enumerate(range(0, n, cfg.frame_length)):
        pk.append(ae.frame(cfg, [c[s:s + cfg.frame_length] for c in chans], [specs[k % len(specs)]]))
    return pk


def _both(tmp_path, cfg, chans, specs):
    pk = _frames(cfg, chans, specs)
    want = ae.expected_mono(cfg, chans)
    x, sr = _decode(tmp_path, ae.caf(cfg, pk, len(chans[0])), "t.caf")
    assert sr == cfg.sample_rate
    assert x.tobytes() == want.tobytes()
    chunks = [1] * len(pk) if len(pk) < 3 else [2] + [1] * (len(pk) - 2)
    x, sr = _decode(tmp_path, ae.mp4(cfg, pk, chunks), "t.m4a")
    assert sr == cfg.sample_rate
    assert x.tobytes() == want.tobytes()


MONO_SPECS = [
    {"ch": [{"coefs": [], "den": 9}]},                                      # numactive 0
    {"ch": [{"na31": True}]},                                               # first-order
    {"ch": [{"coefs": [1024, -512, 256, -128], "den": 9, "pbf": 4}]},       # 4 taps
    {"ch": [{"coefs": [600, 300, -100, 50, 20, -10, 5, 2], "den": 9}]},     # 8 taps
    {"ch": [{"mode": 15, "coefs": [400, -200, 100, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 7], "den": 10,
             "pbf": 2}]},                                                   # mode 15, 16 taps
    {"escape": True},                                                       # raw samples
]


def test_mono_16(tmp_path):
    cfg = ae.Config(bit_depth=16, channels=1, frame_length=1024)
    s = _sig(6 * 1024 + 333, 16, 1, silence=[(2100, 2900), (5000, 5003)])  # zero runs; partial frame
    _both(tmp_path, cfg, [s], MONO_SPECS)


def test_mono_16_large_residuals_escape(tmp_path):
    cfg = ae.Config(bit_depth=16, channels=1, frame_length=512, kb=10)
    rng = np.random.default_rng(5)
    s = rng.integers(-32768, 32768, 2048).astype(np.int64)  # white noise: Golomb escapes
    s[100:110] = [32767, -32768] * 5
    _both(tmp_path, cfg, [s], [{"ch": [{"coefs": [], "den": 9}]}, {"ch": [{"coefs": [512, -256], "den": 9}]}])


@pytest.mark.parametrize("mix", [(0, 0), (2, 1), (2, 2), (3, -2)])
def test_stereo_16(tmp_path, mix):
    cfg = ae.Config(bit_depth=16, channels=2, frame_length=1024, sample_rate=48000)
    l = _sig(3000, 16, 2, amp=0.4)
    r = (0.7 * l + _sig(3000, 16, 3, amp=0.1)).astype(np.int64)
    ch = [{"coefs": [800, -300, 100, 20], "den": 9}, {"coefs": [900, -400], "den": 9, "mode": 15}]
    _both(tmp_path, cfg, [l, r], [{"mix": mix, "ch": ch}, {"escape": True}, {"mix": mix, "ch": ch[::-1]}])


@pytest.mark.parametrize("bits,shift", [(24, 1), (24, 0), (20, 0), (32, 2)])
def test_wide_samples(tmp_path, bits, shift):
    nch = 2 if bits == 24 else 1
    cfg = ae.Config(bit_depth=bits, channels=nch, frame_length=1024)
    chans = [_sig(2500, bits, 7 + c, amp=0.3 if nch == 2 else 0.6) for c in range(nch)]
    ch = [{"coefs": [700, -200, 60, -10], "den": 9}] * nch
    _both(tmp_path, cfg, chans, [{"shift": shift, "mix": (2, 1), "ch": ch}, {"escape": True}])


def test_caf_cookie_wrapper_and_damaged_packet(tmp_path):
    cfg = ae.Config(bit_depth=16, channels=1, frame_length=1024)
    s = _sig(3072, 16, 11)
    pk = _frames(cfg, [s], [{"ch": [{"coefs": [1000, -400], "den": 9}]}])
    x, _ = _decode(tmp_path, ae.caf(cfg, pk, 3072, wrap_cookie=True), "t.caf")
    assert x.tobytes() == ae.expected_mono(cfg, [s]).tobytes()
    bad = bytearray(pk[1])
    bad[0] = 0xA0  # element tag 5 (PCE): not decodable here -> the packet is skipped
    x, _ = _decode(tmp_path, ae.caf(cfg, [pk[0], bytes(bad), pk[2]], 3072), "t.caf")
    want = ae.expected_mono(cfg, [np.concatenate([s[:1024], s[2048:]])])
    assert x.tobytes() == want.tobytes()


def test_mp4_aac_is_named(tmp_path):
    cfg = ae.Config()
    with pytest.raises(sdsp.AnalysisError) as e:
        _decode(tmp_path, ae.mp4(cfg, [b"\x00" * 10], [1], codec=b"mp4a"), "t.m4a")
    assert "AAC" in str(e.value) and e.value.kind == "DecodingError"
