"""A small FLAC encoder for the decode front-end's tests (TEST INFRASTRUCTURE).

The reference decodes FLAC through symphonia 0.5 (Cargo.toml:15, examples/analyze_batch.rs:30-148);
neither symphonia nor a FLAC encoder is in this image, and the reference holds no FLAC fixture,
so the FLAC parity of the native decoder (stratum-dsp_amd/csrc/host_flac.hip) is pinned by
streams written here from the format specification (RFC 9639) and by the examples' published
conversion of symphonia's S32 buffers ("parity unpinned" against symphonia itself).

Every coding choice is explicit so the tests can cover each one: subframe type (CONSTANT,
VERBATIM, FIXED 0-4, LPC with given precision / shift / coefficients), wasted bits, residual
coding method (4- or 5-bit Rice parameters), partition order, escaped partitions, channel
assignment (independent, left/side, side/right, mid/side), block-size and sample-rate codes,
fixed or variable blocking strategy.
"""
import numpy as np


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, k):
        """k low bits of v (two's complement for negative v), most significant first."""
        if k == 0:
            return
        v &= (1 << k) - 1
        self.acc = (self.acc << k) | v
        self.n += k
        while self.n >= 8:
            self.n -= 8
            self.out.append((self.acc >> self.n) & 0xFF)
        self.acc &= (1 << self.n) - 1

    def unary(self, q):
        for _ in range(q):
            self.put(0, 1)
        self.put(1, 1)

    def align(self):
        if self.n:
            self.put(0, 8 - self.n)

    def bytes(self):
        assert self.n == 0
        return bytes(self.out)


def crc8(data):
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data):
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def utf8_number(v):
    """FLAC's UTF-8-like coding of the frame / sample number (up to 36 bits)."""
    if v < 0x80:
        return bytes([v])
    for nbytes, lim in ((2, 1 << 11), (3, 1 << 16), (4, 1 << 21), (5, 1 << 26), (6, 1 << 31), (7, 1 << 36)):
        if v < lim:
            break
    extra = nbytes - 1
    cont = [0x80 | ((v >> (6 * i)) & 0x3F) for i in range(extra)][::-1]
    lead = ((0xFF << (8 - nbytes)) & 0xFF) | (v >> (6 * extra))
    return bytes([lead] + cont)


FIXED_BS = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12,
            8192: 13, 16384: 14, 32768: 15}
RATE_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
              48000: 10, 96000: 11}
BPS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def zigzag(r):
    return 2 * r if r >= 0 else -2 * r - 1


def write_residual(w, res, order, bs, method=0, porder=0, escape=(), params=None):
    """res: residual values for indices order..bs-1.  escape: partition indices written raw."""
    w.put(method, 2)
    w.put(porder, 4)
    pbits = 4 if method == 0 else 5
    esc = (1 << pbits) - 1
    parts = 1 << porder
    i = 0
    for p in range(parts):
        cnt = (bs >> porder) - (order if p == 0 else 0)
        vals = [int(v) for v in res[i:i + cnt]]
        i += cnt
        if p in escape:
            nb = max([0] + [max(v.bit_length() + 1, 1) for v in vals if v != 0])
            w.put(esc, pbits)
            w.put(nb, 5)
            for v in vals:
                w.put(v, nb)
            continue
        if params is not None:
            k = params[p]
        else:
            mean = (sum(zigzag(v) for v in vals) / max(len(vals), 1)) if vals else 0
            k = max(0, int(np.floor(np.log2(mean))) if mean >= 1 else 0)
            k = min(k, esc - 1)
        w.put(k, pbits)
        for v in vals:
            u = zigzag(v)
            w.unary(u >> k)
            w.put(u & ((1 << k) - 1), k)


def fixed_residual(s, order):
    s = [int(v) for v in s]
    r = []
    for i in range(order, len(s)):
        if order == 0:
            p = 0
        elif order == 1:
            p = s[i - 1]
        elif order == 2:
            p = 2 * s[i - 1] - s[i - 2]
        elif order == 3:
            p = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]
        else:
            p = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]
        r.append(s[i] - p)
    return r


def lpc_residual(s, coefs, shift):
    s = [int(v) for v in s]
    order = len(coefs)
    return [s[i] - (sum(c * s[i - 1 - j] for j, c in enumerate(coefs)) >> shift) for i in range(order, len(s))]


def write_subframe(w, s, bps, spec):
    """spec: dict(type=..., order, wasted, method, porder, escape, coefs, prec, shift, params)."""
    s = [int(v) for v in s]
    t = spec.get("type", "fixed")
    wasted = spec.get("wasted", 0)
    if wasted:
        assert all(v % (1 << wasted) == 0 for v in s)
        s = [v >> wasted for v in s]
    wb = bps - wasted
    bs = len(s)
    w.put(0, 1)
    code = {"constant": 0, "verbatim": 1}.get(t)
    if t == "fixed":
        code = 8 + spec["order"]
    elif t == "lpc":
        code = 31 + len(spec["coefs"])
    w.put(code, 6)
    if wasted:
        w.put(1, 1)
        w.unary(wasted - 1)
    else:
        w.put(0, 1)
    if t == "constant":
        assert len(set(s)) == 1
        w.put(s[0], wb)
    elif t == "verbatim":
        for v in s:
            w.put(v, wb)
    elif t == "fixed":
        o = spec["order"]
        for v in s[:o]:
            w.put(v, wb)
        write_residual(w, fixed_residual(s, o), o, bs, spec.get("method", 0), spec.get("porder", 0),
                       spec.get("escape", ()), spec.get("params"))
    else:
        coefs, prec, shift = spec["coefs"], spec["prec"], spec["shift"]
        o = len(coefs)
        for v in s[:o]:
            w.put(v, wb)
        w.put(prec - 1, 4)
        w.put(shift, 5)
        for c in coefs:
            assert -(1 << (prec - 1)) <= c < (1 << (prec - 1))
            w.put(c, prec)
        write_residual(w, lpc_residual(s, coefs, shift), o, bs, spec.get("method", 0), spec.get("porder", 0),
                       spec.get("escape", ()), spec.get("params"))


def frame(chans, bps, number, assign="indep", specs=None, bs_mode="auto", rate=None, rate_mode="stream",
          bps_mode="frame", variable=False):
    """One FLAC frame.  chans: list of int arrays (the original channels, e.g. left/right).
    assign: indep | left_side | side_right | mid_side.  Returns bytes."""
    bs = len(chans[0])
    nch = len(chans)
    if assign == "left_side":
        coded, cbps, chc = [chans[0], [a - b for a, b in zip(chans[0], chans[1])]], [bps, bps + 1], 8
    elif assign == "side_right":
        coded, cbps, chc = [[a - b for a, b in zip(chans[0], chans[1])], chans[1]], [bps + 1, bps], 9
    elif assign == "mid_side":
        coded = [[(int(a) + int(b)) >> 1 for a, b in zip(chans[0], chans[1])],
                 [int(a) - int(b) for a, b in zip(chans[0], chans[1])]]
        cbps, chc = [bps, bps + 1], 10
    else:
        coded, cbps, chc = chans, [bps] * nch, nch - 1
    specs = specs or [{"type": "fixed", "order": 2}] * len(coded)
    h = BitWriter()
    h.put(0x3FFE, 14)
    h.put(0, 1)
    h.put(1 if variable else 0, 1)
    extra_bs = None
    if bs_mode == "auto" and bs in FIXED_BS:
        h.put(FIXED_BS[bs], 4)
    elif bs_mode == "8" or (bs_mode == "auto" and bs <= 256):
        h.put(6, 4)
        extra_bs = (bs - 1, 8)
    else:
        h.put(7, 4)
        extra_bs = (bs - 1, 16)
    extra_sr = None
    if rate_mode == "stream":
        h.put(0, 4)
    elif rate_mode == "code":
        h.put(RATE_CODES[rate], 4)
    elif rate_mode == "khz":
        h.put(12, 4)
        extra_sr = (rate // 1000, 8)
    elif rate_mode == "hz":
        h.put(13, 4)
        extra_sr = (rate, 16)
    else:  # tens of Hz
        h.put(14, 4)
        extra_sr = (rate // 10, 16)
    h.put(chc, 4)
    h.put(0 if bps_mode == "stream" else BPS_CODES[bps], 3)
    h.put(0, 1)
    hb = bytearray(h.bytes()) + utf8_number(number)
    w2 = BitWriter()
    if extra_bs:
        w2.put(*extra_bs)
    if extra_sr:
        w2.put(*extra_sr)
    hb += w2.bytes()
    hb.append(crc8(hb))
    w = BitWriter()
    for c, b, sp in zip(coded, cbps, specs):
        write_subframe(w, c, b, sp)
    w.align()
    body = bytes(hb) + w.bytes()
    return body + crc16(body).to_bytes(2, "big")


def stream(frames, rate, nch, bps, total=0, id3=False):
    si = BitWriter()
    si.put(16, 16)
    si.put(65535, 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(rate, 20)
    si.put(nch - 1, 3)
    si.put(bps - 1, 5)
    si.put(total, 36)
    si.put(0, 64)
    si.put(0, 64)
    meta = bytes([0x00, 0, 0, 34]) + si.bytes()
    pad = bytes([0x81, 0, 0, 5]) + bytes(5)  # a last PADDING block
    head = b""
    if id3:
        body = bytes(20)
        head = b"ID3" + bytes([4, 0, 0, 0, 0, 0, len(body)]) + body
    return head + b"fLaC" + meta + pad + b"".join(frames)


def expected_mono(chan_frames, bps):
    """The reference examples' conversion of symphonia's S32 buffers: (s << (32 - bps)) as f32 /
    2^31 per channel, mono = channel sum from -0.0 in channel order / channels (f32)."""
    out = []
    for chans in chan_frames:
        conv = []
        for c in chans:
            u = (np.asarray(c, dtype=np.int64) << (32 - bps)) & 0xFFFFFFFF
            s32 = u.astype(np.uint32).view(np.int32)
            conv.append(s32.astype(np.float32) / np.float32(2147483648.0))
        if len(conv) == 1:
            out.append(conv[0])
        else:
            acc = np.full(len(conv[0]), np.float32(-0.0), dtype=np.float32)
            for v in conv:
                acc = (acc + v).astype(np.float32)
            out.append((acc / np.float32(len(conv))).astype(np.float32))
    return np.concatenate(out) if out else np.zeros(0, np.float32)
