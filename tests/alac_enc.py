"""A small Apple Lossless (ALAC) encoder and CAF / MP4 writers for the decode front-end's tests
(TEST INFRASTRUCTURE).

The reference decodes ALAC through symphonia (Cargo.toml:15, features = ["all"]); this image has
neither symphonia nor an ALAC encoder and the reference holds no ALAC file, so the streams are
written here from Apple's published ALAC format: the ALACSpecificConfig cookie, frames of SCE /
CPE elements with the adaptive Golomb coder (zero runs, escapes), the sign-adaptive FIR predictor
(prediction modes 0 and 15, numactive 0 / 31 / n), "bytes shifted" low bits, stereo mixing, raw
(escaped) elements and partial frames.  The encoder runs the decoder's own state updates forward,
so every choice below is explicit and the expected PCM is the encoded PCM (ALAC is lossless);
parity against symphonia itself is unpinned.
"""
import struct

import numpy as np

from flac_enc import BitWriter

QBSHIFT, MMULSHIFT, BITOFF, MAX_PREFIX = 9, 2, 24, 9
MDENSHIFT = QBSHIFT - MMULSHIFT - 1
MOFF = 1 << (MDENSHIFT - 2)
M32 = 0xFFFFFFFF


def _clz32(x):
    return 32 - int(x).bit_length() if x else 32


def _sext(v, bits):
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def _i32(v):
    return _sext(v, 32)


def _sign(v):
    return (v > 0) - (v < 0)


class Config:
    def __init__(self, bit_depth=16, channels=1, frame_length=4096, pb=40, mb=10, kb=14, max_run=255,
                 sample_rate=44100):
        self.bit_depth, self.channels, self.frame_length = bit_depth, channels, frame_length
        self.pb, self.mb, self.kb, self.max_run, self.sample_rate = pb, mb, kb, max_run, sample_rate

    def cookie(self):
        return struct.pack(">IBBBBBBHIII", self.frame_length, 0, self.bit_depth, self.pb, self.mb, self.kb,
                           self.channels, self.max_run, 0, 0, self.sample_rate)


def _code(w, x, m, k, escape_bits):
    """One adaptive-Golomb value: pre = x // m ones, a zero, then r + 1 in k bits (r > 0) or
    k - 1 zero bits (r = 0); an escape (9 ones, then x in escape_bits) from pre >= 9."""
    pre, r = divmod(x, m) if m else (MAX_PREFIX, 0)
    if pre >= MAX_PREFIX:
        w.put((1 << MAX_PREFIX) - 1, MAX_PREFIX)
        w.put(x, escape_bits)
        return
    w.put((1 << pre) - 1, pre)
    w.put(0, 1)
    if k == 1:
        return
    if r == 0:
        w.put(0, k - 1)
    else:
        w.put(r + 1, k)


def ag_encode(w, res, cfg, pb_factor, chan_bits):
    """dyn_comp: the inverse of the decoder's dyn_decomp (same state updates)."""
    pb = (cfg.pb * pb_factor) // 4
    wb = (1 << cfg.kb) - 1
    mb, zmode, i, n = cfg.mb, 0, 0, len(res)
    while i < n:
        k = min(31 - _clz32((mb >> QBSHIFT) + 3), cfg.kb)
        m = (1 << k) - 1
        x = int(res[i])
        nd = 2 * x if x >= 0 else -2 * x - 1
        v = nd - zmode
        assert v >= 0, "a zero right after a zero run"
        _code(w, v, m, k, chan_bits)
        i += 1
        mb = (pb * (v + zmode) + mb - ((pb * mb) >> QBSHIFT)) & M32
        if v > 0xFFFF:
            mb = 0xFFFF
        zmode = 0
        if ((mb << MMULSHIFT) & M32) < (1 << QBSHIFT) and i < n:
            zmode = 1
            kz = _clz32(mb) - BITOFF + ((mb + MOFF) >> MDENSHIFT)
            mz = ((1 << kz) - 1) & wb
            run = 0
            while i + run < n and res[i + run] == 0 and run < 65535:
                run += 1
            _code(w, run, mz, kz, 16)
            i += run
            if run >= 65535:
                zmode = 0
            mb = 0


def predict(out, coefs, na, chan_bits, den_shift):
    """Residuals pc with unpc_block(pc) == out; coefs adapt as in the decoder."""
    n = len(out)
    out = [int(v) for v in out]
    pc = [0] * n
    if n == 0:
        return pc
    pc[0] = out[0]
    if na == 0:
        return [out[0]] + out[1:]
    if na == 31:
        for j in range(1, n):
            pc[j] = _sext(out[j] - out[j - 1], chan_bits)
        return pc
    coefs = list(coefs)
    for j in range(1, min(na + 1, n)):
        pc[j] = _sext(out[j] - out[j - 1], chan_bits)
    den_half = 1 << (den_shift - 1) if den_shift > 0 else 0
    lim = na + 1
    for j in range(lim, n):
        top = out[j - lim]
        s = 0
        for k in range(na):
            s = (s + coefs[k] * (out[j - 1 - k] - top)) & M32
        pred = _i32(s + den_half) >> den_shift
        d = _sext(out[j] - top - pred, chan_bits)
        pc[j] = d
        del0, sg = d, _sign(d)
        if sg > 0:
            for k in range(na - 1, -1, -1):
                dd = _i32(top - out[j - 1 - k])
                sgn = _sign(dd)
                coefs[k] = _sext(coefs[k] - sgn, 16)
                del0 -= (na - k) * ((sgn * dd) >> den_shift)
                if del0 <= 0:
                    break
        elif sg < 0:
            for k in range(na - 1, -1, -1):
                dd = _i32(top - out[j - 1 - k])
                sgn = _sign(dd)
                coefs[k] = _sext(coefs[k] + sgn, 16)
                del0 -= (na - k) * ((-sgn * dd) >> den_shift)
                if del0 >= 0:
                    break
    return pc


def element(w, cfg, chans, spec):
    """One SCE (1 channel) or CPE (2) element of a frame.  spec: escape, shift (bytes), partial,
    mix (bits, res), and per channel mode (0 / 15), coefs, den_shift, pb_factor."""
    ech = len(chans)
    n = len(chans[0])
    shift = 8 * spec.get("shift", 0)
    escape = spec.get("escape", False)
    partial = n != cfg.frame_length
    w.put(1 if ech == 2 else 0, 3)
    w.put(0, 4)
    w.put(0, 12)
    w.put((int(partial) << 3) | ((0 if escape else shift // 8) << 1) | int(escape), 4)
    if partial:
        w.put(n >> 16, 16)
        w.put(n & 0xFFFF, 16)
    bits = cfg.bit_depth
    if escape:
        for i in range(n):
            for c in chans:
                v = int(c[i])
                if bits <= 16:
                    w.put(v, bits)
                else:
                    w.put(v >> (bits - 16), 16)
                    w.put(v & ((1 << (bits - 16)) - 1), bits - 16)
        return
    chan_bits = bits - shift + (1 if ech == 2 else 0)
    hi = [[int(v) >> shift for v in c] for c in chans]
    lo = [[int(v) & ((1 << shift) - 1) for v in c] for c in chans]
    if ech == 2:
        mix_bits, mix_res = spec.get("mix", (0, 0))
        L, R = hi
        v = [a - b for a, b in zip(L, R)]
        u = [b + ((mix_res * d) >> mix_bits) if mix_res else a for a, b, d in zip(L, R, v)]
        if not mix_res:
            u, v = L, R
        mixed = [u, v]
        w.put(mix_bits, 8)
        w.put(mix_res & 0xFF, 8)
    else:
        mixed = hi
    chs = spec.get("ch", [{}] * ech)
    def coefs_of(c):  # numactive 31 (first-order prediction) still carries 31 coefficients
        return [0] * 31 if c.get("na31") else list(c.get("coefs", []))

    for e in range(ech):
        c = chs[e]
        coefs = coefs_of(c)
        w.put((c.get("mode", 0) << 4) | c.get("den", 9), 8)
        w.put((c.get("pbf", 4) << 5) | len(coefs), 8)
        for q in coefs:
            w.put(q, 16)
    if shift:
        for i in range(n):
            for e in range(ech):
                w.put(lo[e][i], shift)
    for e in range(ech):
        c = chs[e]
        coefs = coefs_of(c)
        na = len(coefs)
        src = [_sext(x, chan_bits) for x in mixed[e]]
        if c.get("mode", 0) == 15:
            res = predict_chain(src, coefs, na, chan_bits, c.get("den", 9))
        else:
            res = predict(src, coefs, na, chan_bits, c.get("den", 9))
        ag_encode(w, res, cfg, c.get("pbf", 4), chan_bits)


def predict_chain(out, coefs, na, chan_bits, den):
    """Mode 15: the decoder runs a first-order pass (numactive 31) and then the FIR predictor, so
    the encoder inverts the FIR first and the first-order pass second."""
    mid = predict(out, coefs, na, chan_bits, den)
    return predict(mid, [], 31, chan_bits, 0)


def frame(cfg, chans, specs):
    """A packet: the elements (one spec per element: SCE for 1 channel, CPE for 2), END, padding."""
    w = BitWriter()
    if cfg.channels == 1:
        element(w, cfg, [chans[0]], specs[0])
    else:
        element(w, cfg, [chans[0], chans[1]], specs[0])
    w.put(7, 3)
    w.put(0, (8 - w.n) % 8)  # byte alignment
    return w.bytes()


def _vlq(v):
    out = [v & 0x7F]
    v >>= 7
    while v:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    return bytes(reversed(out))


def caf(cfg, packets, frames_total, wrap_cookie=False):
    desc = struct.pack(">d", float(cfg.sample_rate)) + b"alac" + struct.pack(">IIIII", 0, 0, cfg.frame_length,
                                                                              cfg.channels, 0)
    kuki = cfg.cookie()
    if wrap_cookie:
        kuki = struct.pack(">I", 12) + b"frma" + b"alac" + struct.pack(">I", 36) + b"alac" + bytes(4) + kuki
    pakt = struct.pack(">qqii", len(packets), frames_total, 0, 0) + b"".join(_vlq(len(p)) for p in packets)
    data = struct.pack(">I", 0) + b"".join(packets)
    out = b"caff" + struct.pack(">HH", 1, 0)
    for cid, body in [(b"desc", desc), (b"kuki", kuki), (b"pakt", pakt), (b"data", data)]:
        out += cid + struct.pack(">q", len(body)) + body
    return out


def _box(t, body):
    return struct.pack(">I", 8 + len(body)) + t + body


def mp4(cfg, packets, chunks, codec=b"alac"):
    """ISO MP4 with one audio track; `chunks` = samples per chunk, in order (stsc runs)."""
    ftyp = _box(b"ftyp", b"M4A " + struct.pack(">I", 0) + b"M4A mp42isom")
    entry_body = bytes(6) + struct.pack(">H", 1) + struct.pack(">HHIHHHHI", 0, 0, 0, cfg.channels, cfg.bit_depth, 0, 0,
                                                             cfg.sample_rate << 16)
    if codec == b"alac":
        entry_body += _box(b"alac", bytes(4) + cfg.cookie())
    stsd = _box(b"stsd", struct.pack(">II", 0, 1) + _box(codec, entry_body))
    stsz = _box(b"stsz", struct.pack(">III", 0, 0, len(packets)) + b"".join(struct.pack(">I", len(p)) for p in packets))
    runs = []
    for i, c in enumerate(chunks):
        if not runs or runs[-1][1] != c:
            runs.append((i + 1, c))
    stsc = _box(b"stsc", struct.pack(">II", 0, len(runs)) + b"".join(struct.pack(">III", a, b, 1) for a, b in runs))

    def build(offsets):
        stco = _box(b"stco", struct.pack(">II", 0, len(offsets)) + b"".join(struct.pack(">I", o) for o in offsets))
        stbl = _box(b"stbl", stsd + _box(b"stts", struct.pack(">II", 0, 0)) + stsc + stsz + stco)
        minf = _box(b"minf", _box(b"smhd", bytes(8)) + stbl)
        hdlr = _box(b"hdlr", bytes(8) + b"soun" + bytes(12) + b"\0")
        mdia = _box(b"mdia", _box(b"mdhd", bytes(24)) + hdlr + minf)
        trak = _box(b"trak", _box(b"tkhd", bytes(84)) + mdia)
        return _box(b"moov", _box(b"mvhd", bytes(100)) + trak)

    moov = build([0] * len(chunks))
    base = len(ftyp) + len(moov) + 8
    offsets, pos, k = [], base, 0
    for c in chunks:
        offsets.append(pos)
        for _ in range(c):
            pos += len(packets[k])
            k += 1
    moov = build(offsets)
    return ftyp + moov + _box(b"mdat", b"".join(packets))


def expected_mono(cfg, chans):
    """The examples' conversion of the decoded integers: / 2^(bits - 1) (/ 32768 at 16 bits,
    / 2^31 at 32), channels summed from -0.0 in order, / channels."""
    scale = np.float32(2.0 ** (cfg.bit_depth - 1))
    conv = [np.asarray(c, np.int64).astype(np.float32) / scale for c in chans]
    if len(conv) == 1:
        return conv[0]
    acc = np.full(len(conv[0]), np.float32(-0.0), np.float32)
    for v in conv:
        acc = (acc + v).astype(np.float32)
    return (acc / np.float32(len(conv))).astype(np.float32)
