"""Ogg Vorbis (stratum-dsp_amd/csrc/host_vorbis.hip) through the C ABI (sdsp_decode_audio_file),
on the CPU.

The reference decodes Vorbis through symphonia (Cargo.toml:15, features = ["all"]) and mixes its
f32 buffers to mono (examples/analyze_file.rs:25-180).  The streams are written by
tests/vorbis_enc.py from the Vorbis I specification; the expected samples are the encoder's own
float32 synthesis of its quantised spectra (inverse coupling, floor x residue, the inverse MDCT by
its defining sum, the windows, the overlap-add), so the check covers the bitstream decode exactly
and the transform to within float32 rounding.  The decoded signal must also track the encoded
one (a lossy codec: a loose bound).  Parity against symphonia itself is unpinned.
"""
import os

import numpy as np
import pytest

import sdsp
import vorbis_enc as ve

F32 = np.float32


def _sig(n, seed, nch):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 44100
    out = []
    for c in range(nch):
        x = 0.4 * np.sin(2 * np.pi * (220 + 110 * c) * t) + 0.2 * np.sin(2 * np.pi * 1375 * t)
        x += 0.02 * rng.standard_normal(n)
        x[n // 3:n // 3 + 300] += 0.5 * np.sin(2 * np.pi * 3000 * t[:300])  # a transient burst
        out.append(x)
    return out


def _decode(tmp_path, data):
    p = tmp_path / "t.ogg"
    p.write_bytes(data)
    return sdsp.decode_audio_file(str(p))


def _mono(chans):
    if len(chans) == 1:
        return chans[0].astype(F32)
    acc = np.full(len(chans[0]), F32(-0.0), F32)
    for c in chans:
        acc = (acc + c.astype(F32)).astype(F32)
    return (acc / F32(len(chans))).astype(F32)


def _run(tmp_path, nch, pattern, rtype, silent=(), final_cut=0):
    bs = [256, 2048]
    span = sum(bs[pattern[k - 1]] // 4 + bs[pattern[k]] // 4 for k in range(1, len(pattern)))
    x = _sig(span, 3 + nch + rtype, nch)
    pk, gr, exp = ve.encode(x, 44100, pattern, rtype=rtype, silent_blocks=silent)
    final = gr[-1] - final_cut if final_cut else None
    data = ve.ogg_stream(ve.headers(nch, 44100, rtype), pk, gr, final_len=final)
    got, sr = _decode(tmp_path, data)
    want = _mono(exp)
    if final_cut:
        want = want[:len(want) - final_cut]
    assert sr == 44100
    assert got.shape == want.shape
    tol = 2e-6 * max(1.0, float(np.max(np.abs(want))))
    assert float(np.max(np.abs(got - want))) <= tol
    return got, _mono([c[:len(want)] for c in x]), want


PATTERNS = {
    "long": [1] * 8,
    "short": [0] * 24,
    "mixed": [1, 1, 0, 0, 0, 1, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1],
}


@pytest.mark.parametrize("rtype", [0, 1, 2])
@pytest.mark.parametrize("pattern", sorted(PATTERNS))
def test_vorbis_mono(tmp_path, rtype, pattern):
    got, orig, _ = _run(tmp_path, 1, PATTERNS[pattern], rtype)
    # the codec tracks its input (quantisation against the floor only: ~12 % RMS with short blocks)
    err = np.sqrt(np.mean((got - orig) ** 2))
    assert err < 0.2 * np.sqrt(np.mean(orig ** 2)), err


@pytest.mark.parametrize("rtype", [1, 2])
def test_vorbis_stereo_coupled(tmp_path, rtype):
    got, orig, _ = _run(tmp_path, 2, PATTERNS["mixed"], rtype)
    err = np.sqrt(np.mean((got - orig) ** 2))
    assert err < 0.3 * np.sqrt(np.mean(orig ** 2)), err


def test_vorbis_unused_floor_and_granule_cut(tmp_path):
    # block 3 codes an unused floor (silence); the last page's granule cuts 100 samples
    _run(tmp_path, 1, PATTERNS["long"], 1, silent=(3,), final_cut=100)


def test_vorbis_errors(tmp_path):
    hdr = ve.headers(1, 44100, 1)
    with pytest.raises(sdsp.AnalysisError) as e:
        _decode(tmp_path, ve.ogg_stream(hdr[:2], [], []))
    assert e.value.kind == "DecodingError"
    bad = bytearray(hdr[2])
    bad[8] ^= 0xFF  # the first codebook's sync pattern
    with pytest.raises(sdsp.AnalysisError) as e:
        _decode(tmp_path, ve.ogg_stream([hdr[0], hdr[1], bytes(bad)], [b"\x00"], [0]))
    assert "Vorbis" in str(e.value)


@pytest.mark.parametrize("damage", ["mux", "dup_x", "big_dims"])
def test_vorbis_malformed_setup_rejected(tmp_path, damage):
    """Setup headers the Vorbis I specification forbids fail with a decoding error instead of
    reading out of bounds: a channel mux naming a submap that does not exist (§4.2.4), a floor-1 X
    list with a repeated value (§7.2.2; the curve would divide by zero), and a type-2 lookup whose
    entries x dimensions is 2^32 (0 in 32-bit arithmetic; the value table would be 16 GB)."""
    hdr = ve.headers(1, 44100, 1, damage=damage)
    pk, gr, _ = ve.encode(_sig(4096, 5, 1), 44100, [1, 1, 1], rtype=1)
    with pytest.raises(sdsp.AnalysisError) as e:
        _decode(tmp_path, ve.ogg_stream(hdr, pk, gr))
    assert e.value.kind == "DecodingError" and "Vorbis" in str(e.value), str(e.value)


REAL_OGG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "real_libvorbis_keypress.ogg")


def test_vorbis_real_libvorbis_stream():
    """A stream from a real encoder (tests/golden/real_libvorbis_keypress.ogg: MathJax's
    a11y/invalid_keypress.ogg, Apache-2.0, vendor string "Xiph.Org libVorbis I 20070622"): its
    codebooks, floors, residues and block switching are libvorbis's, not tests/vorbis_enc.py's.
    No reference decode ships with it, so the checks are properties of a correct decode: the
    stream's length and rate, a smooth waveform (a misdecoded floor, residue or window shows as a
    click at a block edge), the 156 Hz buzz the file holds, then silence."""
    x, sr = sdsp.decode_audio_file(REAL_OGG)
    assert sr == 44100 and len(x) == 22050
    assert np.all(np.isfinite(x)) and 0.3 < float(np.max(np.abs(x))) < 1.0
    assert float(np.max(np.abs(np.diff(x)))) < 0.05
    spec = np.abs(np.fft.rfft(x * np.hanning(len(x))))
    f0 = float(np.fft.rfftfreq(len(x), 1.0 / sr)[np.argmax(spec)])
    assert abs(f0 - 156.0) < 4.0, f0
    head, tail = x[:8192], x[12288:]
    assert float(np.sqrt(np.mean(head ** 2))) > 0.1 and float(np.sqrt(np.mean(tail ** 2))) < 1e-3
