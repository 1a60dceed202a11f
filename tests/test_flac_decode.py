"""The decode front-end's FLAC path (stratum-dsp_amd/csrc/host_flac.hip) through the C ABI
(sdsp_decode_audio_file), on the CPU.

The reference decodes FLAC with symphonia 0.5 and converts its S32 buffers as
examples/analyze_batch.rs:30-177 shows; this image has neither symphonia nor a FLAC encoder and
the reference ships no FLAC fixture, so the streams are written by tests/flac_enc.py from the
format specification and the expected samples follow the examples' conversion (parity against
symphonia itself is unpinned).  Covered: every subframe type, FIXED orders 0-4, LPC orders 1-32
with several precisions / shifts, wasted bits, both Rice parameter widths, partition orders,
escaped partitions, all stereo decorrelations, 1-8 channels, 8/12/16/20/24/32-bit samples,
every block-size and sample-rate code form, fixed and variable blocking, an ID3v2 prefix, a
frame with a bad CRC (skipped, as the examples skip a packet that fails to decode), and the
errors.
"""
import numpy as np
import pytest

import flac_enc as fe
import sdsp


def _signal(n, bps, seed, step=1):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    amp = (1 << (bps - 1)) - 1
    x = 0.6 * np.sin(2 * np.pi * t * (220 + 30 * seed) / 44100) + 0.2 * rng.standard_normal(n) * 0.3
    v = np.clip(np.round(x * amp), -amp - 1, amp).astype(np.int64)
    return (v // step) * step


def _decode(tmp_path, data, name="t.flac"):
    p = tmp_path / name
    p.write_bytes(data)
    return sdsp.decode_audio_file(str(p))


def _check(tmp_path, frames_chans, bps, frames, rate=44100, nch=None, id3=False):
    nch = nch or len(frames_chans[0])
    data = fe.stream(frames, rate, nch, bps, total=sum(len(c[0]) for c in frames_chans), id3=id3)
    x, sr = _decode(tmp_path, data)
    want = fe.expected_mono(frames_chans, bps)
    assert sr == rate
    assert x.dtype == np.float32 and x.shape == want.shape
    assert x.tobytes() == want.tobytes()
    return x


@pytest.mark.parametrize("order", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("method", [0, 1])
def test_fixed_orders(tmp_path, order, method):
    bps = 16
    frames, chans = [], []
    for k, porder in enumerate([0, 2, 4]):
        s = _signal(4096, bps, 10 + k)
        chans.append([s])
        frames.append(fe.frame([s], bps, k, specs=[{"type": "fixed", "order": order, "method": method,
                                                     "porder": porder}]))
    _check(tmp_path, chans, bps, frames)


@pytest.mark.parametrize("order,prec,shift", [(1, 12, 10), (2, 15, 13), (8, 12, 9), (12, 14, 11), (32, 15, 14)])
def test_lpc(tmp_path, order, prec, shift):
    bps = 24
    rng = np.random.default_rng(order)
    coefs = [int(c) for c in rng.integers(-(1 << (prec - 2)), 1 << (prec - 2), size=order)]
    coefs[0] = (1 << shift) - 1  # a dominant first tap keeps the residual informative
    s = _signal(4608, bps, order)
    frames = [fe.frame([s], bps, 0, specs=[{"type": "lpc", "coefs": coefs, "prec": prec, "shift": shift,
                                            "method": 1, "porder": 3}])]
    _check(tmp_path, [[s]], bps, frames)


def test_constant_verbatim_escape_wasted(tmp_path):
    bps = 16
    c = np.full(1152, -1234, np.int64)
    v = _signal(1152, bps, 3)
    e = _signal(2304, bps, 4)
    w = _signal(2304, bps, 5, step=8)  # 3 wasted bits
    frames = [
        fe.frame([c], bps, 0, specs=[{"type": "constant"}]),
        fe.frame([v], bps, 1, specs=[{"type": "verbatim"}]),
        fe.frame([e], bps, 2, specs=[{"type": "fixed", "order": 2, "porder": 2, "escape": (0, 3)}]),
        fe.frame([w], bps, 3, specs=[{"type": "fixed", "order": 1, "wasted": 3}]),
        fe.frame([w], bps, 4, specs=[{"type": "verbatim", "wasted": 3}]),
        fe.frame([np.zeros(576, np.int64)], bps, 5, specs=[{"type": "fixed", "order": 0, "escape": (0,)}]),
    ]
    _check(tmp_path, [[c], [v], [e], [w], [w], [np.zeros(576, np.int64)]], bps, frames)


@pytest.mark.parametrize("assign", ["indep", "left_side", "side_right", "mid_side"])
@pytest.mark.parametrize("bps", [16, 24])
def test_stereo_decorrelation(tmp_path, assign, bps):
    frames, chans = [], []
    for k in range(3):
        left = _signal(2048, bps, 20 + k)
        right = _signal(2048, bps, 40 + k)
        if k == 2:  # full-scale opposite extremes: the side channel needs bps + 1 bits
            left[:8] = (1 << (bps - 1)) - 1
            right[:8] = -(1 << (bps - 1))
        chans.append([left, right])
        frames.append(fe.frame([left, right], bps, k, assign=assign,
                               specs=[{"type": "fixed", "order": 2, "porder": 1}, {"type": "lpc", "coefs": [3, -1],
                                                                                  "prec": 6, "shift": 1}]))
    _check(tmp_path, chans, bps, frames)


@pytest.mark.parametrize("bps", [8, 12, 20, 32])
def test_sample_sizes(tmp_path, bps):
    s = _signal(1024, bps, bps)
    s[:4] = [(1 << (bps - 1)) - 1, -(1 << (bps - 1)), 0, -1]
    frames = [fe.frame([s], bps, 0, specs=[{"type": "verbatim"}]),
              fe.frame([s], bps, 1, specs=[{"type": "fixed", "order": 1, "method": 1}], bps_mode="stream")]
    _check(tmp_path, [[s], [s]], bps, frames)


@pytest.mark.parametrize("nch", [3, 6, 8])
def test_many_channels(tmp_path, nch):
    chans = [_signal(576, 16, 60 + c) for c in range(nch)]
    frames = [fe.frame(chans, 16, 0, specs=[{"type": "fixed", "order": c % 5} for c in range(nch)])]
    _check(tmp_path, [chans], 16, frames)


def test_block_size_and_rate_codes(tmp_path):
    bps = 16
    sizes = [192, 576, 1152, 2304, 4608, 256, 512, 1024, 2048, 4096, 8192, 16384, 100, 7000]
    modes = ["stream", "code", "khz", "hz", "tens"]
    frames, chans, pos = [], [], 0
    for k, n in enumerate(sizes):
        s = _signal(n, bps, 80 + k)
        chans.append([s])
        frames.append(fe.frame([s], bps, pos, variable=True, rate=48000, rate_mode=modes[k % len(modes)],
                               specs=[{"type": "fixed", "order": 2, "porder": 0}]))
        pos += n  # variable blocking: the header carries the first sample's number (UTF-8, up to 3 bytes here)
    # 8-bit and 16-bit explicit block sizes for sizes that also have a table code
    s = _signal(256, bps, 99)
    chans.append([s])
    frames.append(fe.frame([s], bps, pos, variable=True, bs_mode="8", rate=48000))
    s2 = _signal(4096, bps, 98)
    chans.append([s2])
    frames.append(fe.frame([s2], bps, pos + 256, variable=True, bs_mode="16", rate=48000))
    _check(tmp_path, chans, bps, frames, rate=48000)


def test_large_frame_numbers(tmp_path):
    s = _signal(192, 16, 7)
    nums = [0x7F, 0x80, 0x7FF, 0x800, 0xFFFF, 0x10000, 0x1FFFFF, 0x200000, 0x3FFFFFF, 0x4000000, 0x7FFFFFFF]
    frames = [fe.frame([s], 16, v, specs=[{"type": "verbatim"}]) for v in nums]
    _check(tmp_path, [[s]] * len(nums), 16, frames)


def test_bad_crc_frame_is_skipped(tmp_path):
    bps = 16
    a, b, c = _signal(1152, bps, 1), _signal(1152, bps, 2), _signal(1152, bps, 3)
    fa, fb, fc = (fe.frame([x], bps, k, specs=[{"type": "verbatim"}]) for k, x in enumerate((a, b, c)))
    fb = bytearray(fb)
    fb[len(fb) // 2] ^= 0x10  # corrupt the body: the frame CRC-16 no longer matches
    data = fe.stream([fa, bytes(fb), fc], 44100, 1, bps)
    x, _ = _decode(tmp_path, data)
    assert x.tobytes() == fe.expected_mono([[a], [c]], bps).tobytes()


def test_id3_prefix_and_trailing_garbage(tmp_path):
    s = _signal(2048, 16, 11)
    frames = [fe.frame([s], 16, 0)]
    data = fe.stream(frames, 22050, 1, 16, id3=True) + b"\x00\x01garbage"
    x, sr = _decode(tmp_path, data)
    assert sr == 22050 and x.tobytes() == fe.expected_mono([[s]], 16).tobytes()


def test_flac_errors(tmp_path):
    for name, data in [("notflac.flac", b"fLaX" + bytes(40)), ("trunc.flac", b"fLaC\x00\x00\x00\x22" + bytes(10)),
                       ("nosi.flac", b"fLaC" + bytes([0x81, 0, 0, 4]) + bytes(4))]:
        with pytest.raises(sdsp.AnalysisError) as e:
            _decode(tmp_path, data, name)
        assert "Decoding error" in str(e.value)


def test_flac_matches_wav_of_the_same_pcm(tmp_path):
    """The same 16-bit stereo PCM as RIFF/WAVE and as FLAC decodes to the same mono f32 (S16
    `/ 32768` and S32 `<< 16 / 2^31` agree exactly)."""
    import wave

    left, right = _signal(44100, 16, 70), _signal(44100, 16, 71)
    pcm = np.stack([left, right], axis=1).astype("<i2")
    wp = tmp_path / "s.wav"
    with wave.open(str(wp), "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(44100)
        w.writeframes(pcm.tobytes())
    xw, srw = sdsp.decode_audio_file(str(wp))
    frames, chans = [], []
    for k, o in enumerate(range(0, 44100, 4096)):
        l_, r_ = left[o:o + 4096], right[o:o + 4096]
        chans.append([l_, r_])
        frames.append(fe.frame([l_, r_], 16, k, assign="mid_side"))
    xf, srf = _decode(tmp_path, fe.stream(frames, 44100, 2, 16))
    assert srw == srf == 44100 and xw.tobytes() == xf.tobytes()
