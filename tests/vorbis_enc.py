"""A small Ogg Vorbis encoder for the decode front-end's tests (TEST INFRASTRUCTURE).

The reference decodes Vorbis through symphonia (Cargo.toml:15, features = ["all"]); this image has
neither symphonia nor a Vorbis encoder and the reference holds no Vorbis file, so the streams are
written here from the Vorbis I specification, with every choice explicit: short (256) and long
(2048) blocks in any order (the window transitions follow), floor type 1 with a plain class and a
class with a master book and an unused sub-book, residue types 0, 1 and 2 with a silent and an
active classification, a lattice VQ book (lookup type 1, 2 dimensions), square-polar coupling of
a stereo pair, and an unused floor (a silent block).  The encoder computes the floor curves with
the specification's synthesis, quantises the MDCT spectrum against them, and returns, beside the
stream, its own float32 synthesis of what a decoder reconstructs (inverse coupling, floor x
residue, the inverse MDCT by its defining sum, windows, overlap-add): the tests compare the native
decoder with it.  Parity with symphonia itself is unpinned.
"""
import struct

import numpy as np

F32 = np.float32


class LBitWriter:
    """LSB-first bit packing (Vorbis)."""

    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, k):
        v &= (1 << k) - 1 if k else 0
        self.acc |= v << self.n
        self.n += k
        while self.n >= 8:
            self.out.append(self.acc & 0xFF)
            self.acc >>= 8
            self.n -= 8

    def code(self, word, length):
        """A Huffman codeword: its most significant bit first."""
        for b in range(length - 1, -1, -1):
            self.put((word >> b) & 1, 1)

    def bytes(self):
        out = bytes(self.out)
        if self.n:
            out += bytes([self.acc & 0xFF])
        return out


def ilog(v):
    return int(v).bit_length()


def make_words(lengths):
    """The specification's codeword assignment (lowest available codeword per length, in order)."""
    marker = [0] * 33
    words = [None] * len(lengths)
    for i, ln in enumerate(lengths):
        if ln <= 0:
            continue
        entry = marker[ln]
        assert not (ln < 32 and (entry >> ln)), "overspecified"
        words[i] = entry
        for j in range(ln, 0, -1):
            if marker[j] & 1:
                marker[j] = marker[1] + 1 if j == 1 else marker[j - 1] << 1
                break
            marker[j] += 1
        for j in range(ln + 1, 33):
            if (marker[j] >> 1) == entry:
                entry = marker[j]
                marker[j] = marker[j - 1] << 1
            else:
                break
    return words


def float32_pack(v):
    if v == 0:
        return 0
    sign = 0x80000000 if v < 0 else 0
    m, e = abs(v), 0
    mant = m
    while mant < (1 << 20):
        mant *= 2
        e -= 1
    while mant >= (1 << 21):
        mant /= 2
        e += 1
    assert mant == int(mant)
    return sign | ((e + 788) << 21) | int(mant)


class Book:
    def __init__(self, lengths, dims=1, lookup=None):
        self.lengths = lengths
        self.dims = dims
        self.lookup = lookup  # (min, delta, value_bits, lookup_values) for lookup type 1
        self.words = make_words(lengths)

    def write_header(self, w):
        w.put(0x564342, 24)
        w.put(self.dims, 16)
        w.put(len(self.lengths), 24)
        w.put(0, 1)  # unordered
        w.put(0, 1)  # not sparse
        for ln in self.lengths:
            w.put(ln - 1, 5)
        if self.lookup is None:
            w.put(0, 4)
            return
        mn, dl, vbits, nval = self.lookup
        w.put(1, 4)
        w.put(float32_pack(mn), 32)
        w.put(float32_pack(dl), 32)
        w.put(vbits - 1, 4)
        w.put(0, 1)  # sequence_p
        for m in range(nval):
            w.put(m, vbits)

    def emit(self, w, entry):
        w.code(self.words[entry], self.lengths[entry])


def _complete_lengths(n, short):
    """n codeword lengths forming a complete tree: a of `short` bits, the rest of short + 1."""
    a = (1 << (short + 1)) - n
    assert 0 <= a <= n
    return [short] * a + [short + 1] * (n - a)


VQ_VALUES = 65  # lattice values -32 .. 32 per dimension
BOOK_Y = Book([7] * 128)                                  # floor Y values 0 .. 127 (multiplier 2)
BOOK_CLASS = Book([1, 1])                                 # residue classification (silent, active)
BOOK_VQ = Book(_complete_lengths(VQ_VALUES ** 2, 12), dims=2, lookup=(-32.0, 1.0, 7, VQ_VALUES))
BOOK_MASTER = Book([2, 2, 2, 2])                          # floor class with one sub-class bit per dim
BOOKS = [BOOK_Y, BOOK_CLASS, BOOK_VQ, BOOK_MASTER]


class FloorSpec:
    def __init__(self, rangebits, xs):
        self.rangebits = rangebits
        self.X = [0, 1 << rangebits] + xs  # partition 0 (class 0): xs[0:2]; partition 1 (class 1): xs[2:4]


FLOORS = [FloorSpec(7, [16, 48, 80, 104]), FloorSpec(10, [64, 200, 500, 800])]
RANGE = 128  # multiplier 2


def _write_floor(w, f):
    w.put(1, 16)
    w.put(2, 5)           # partitions
    w.put(0, 4)
    w.put(1, 4)           # classes 0, 1
    w.put(1, 3)           # class 0: 2 dims
    w.put(0, 2)           #   no sub-classes
    w.put(0 + 1, 8)       #   sub-book 0 = BOOK_Y
    w.put(1, 3)           # class 1: 2 dims
    w.put(1, 2)           #   1 sub-class bit
    w.put(3, 8)           #   master book BOOK_MASTER
    w.put(0, 8)           #   sub-class 0: no book (Y = 0)
    w.put(0 + 1, 8)       #   sub-class 1: BOOK_Y
    w.put(1, 2)           # multiplier 2
    w.put(f.rangebits, 4)
    for x in f.X[2:]:
        w.put(x, f.rangebits)


def _render_line(x0, y0, x1, y1, v):
    dy, adx = y1 - y0, x1 - x0
    ady = abs(dy)
    base = int(dy / adx)  # C division (toward zero)
    sy = base - 1 if dy < 0 else base + 1
    ady -= abs(base) * adx
    x, y, err = x0, y0, 0
    if x < len(v):
        v[x] = y
    for x in range(x0 + 1, x1):
        err += ady
        if err >= adx:
            err -= adx
            y += sy
        else:
            y += base
        if x < len(v):
            v[x] = y


def inverse_db(i):
    return F32(10.0 ** (-(255 - i) * (140.0 / 256.0) / 20.0))


def floor_synthesis(f, Y, n2):
    """Steps 1 and 2 of floor 1 synthesis (specification), from the coded values Y."""
    X = f.X
    nv = len(X)
    fy = [0] * nv
    used = [False] * nv
    fy[0], fy[1] = Y[0], Y[1]
    used[0] = used[1] = True
    for i in range(2, nv):
        lo = max((j for j in range(i) if X[j] < X[i]), key=lambda j: X[j])
        hi = min((j for j in range(i) if X[j] > X[i]), key=lambda j: X[j])
        pred = _render_point(X[lo], fy[lo], X[hi], fy[hi], X[i])
        val = Y[i]
        highroom, lowroom = RANGE - pred, pred
        room = min(highroom, lowroom) * 2
        if val:
            used[lo] = used[hi] = used[i] = True
            if val >= room:
                fy[i] = val - lowroom + pred if highroom > lowroom else pred - val + highroom - 1
            else:
                fy[i] = pred - (val + 1) // 2 if val & 1 else pred + val // 2
        else:
            fy[i] = pred
    order = sorted(range(nv), key=lambda i: X[i])
    iv = [0] * n2
    lx, ly, hx, hy = 0, fy[order[0]] * 2, 0, 0
    for i in order[1:]:
        if not used[i]:
            continue
        hy, hx = fy[i] * 2, X[i]
        if lx < n2:
            _render_line(lx, ly, hx, hy, iv)
        lx, ly = hx, hy
    if hx < n2:
        _render_line(hx, hy, n2, hy, iv)
    return np.array([inverse_db(min(255, max(0, v))) for v in iv], F32)


def _render_point(x0, y0, x1, y1, x):
    dy, adx = y1 - y0, x1 - x0
    off = abs(dy) * (x - x0) // adx
    return y0 - off if dy < 0 else y0 + off


def floor_values(f, targets):
    """Coded Y values whose synthesis puts each point at its target (0 .. 127) as closely as the
    coding allows; the encoder keeps what the decoder will compute."""
    X = f.X
    nv = len(X)
    Y = [0] * nv
    fy = [0] * nv
    Y[0] = fy[0] = int(targets[0])
    Y[1] = fy[1] = int(targets[1])
    for i in range(2, nv):
        lo = max((j for j in range(i) if X[j] < X[i]), key=lambda j: X[j])
        hi = min((j for j in range(i) if X[j] > X[i]), key=lambda j: X[j])
        pred = _render_point(X[lo], fy[lo], X[hi], fy[hi], X[i])
        t = int(targets[i])
        highroom, lowroom = RANGE - pred, pred
        m = min(highroom, lowroom)
        if t == pred:
            val = 0
        elif t > pred:
            d = t - pred
            val = 2 * d if d < m else d + lowroom
        else:
            d = pred - t
            val = 2 * d - 1 if d <= m else d + highroom - 1
        val = min(val, 127)
        Y[i] = val
        if val:
            room = m * 2
            if val >= room:
                fy[i] = val - lowroom + pred if highroom > lowroom else pred - val + highroom - 1
            else:
                fy[i] = pred - (val + 1) // 2 if val & 1 else pred + val // 2
        else:
            fy[i] = pred
    return Y


def _write_floor_packet(w, Y):
    w.put(1, 1)  # nonzero
    w.put(Y[0], 7)
    w.put(Y[1], 7)
    BOOK_Y.emit(w, Y[2])  # partition 0, class 0: both values through BOOK_Y
    BOOK_Y.emit(w, Y[3])
    cval = (1 if Y[4] else 0) | ((1 if Y[5] else 0) << 1)  # partition 1, class 1: sub-class per dim
    BOOK_MASTER.emit(w, cval)
    for y in (Y[4], Y[5]):
        if y:
            BOOK_Y.emit(w, y)


def vwin(n_len, right):
    i = np.arange(n_len)
    x = (i + 0.5) / n_len * np.pi / 2 + (np.pi / 2 if right else 0.0)
    return np.sin(np.pi / 2 * np.sin(x) ** 2)


def window(n, bs0, blockflag, prev_long, next_long):
    w = np.zeros(n)
    if blockflag and not prev_long:
        ls, ln = n // 4 - bs0 // 4, bs0 // 2
    else:
        ls, ln = 0, n // 2
    if blockflag and not next_long:
        rs, rn = n * 3 // 4 - bs0 // 4, bs0 // 2
    else:
        rs, rn = n // 2, n // 2
    w[ls:ls + ln] = vwin(ln, False)
    w[ls + ln:rs] = 1.0
    w[rs:rs + rn] = vwin(rn, True)
    return w.astype(F32)


def _cos_matrix(n):
    k = np.arange(n // 2)
    t = np.arange(n)
    return np.cos(2 * np.pi / n * (t[:, None] + 0.5 + n / 4) * (k[None, :] + 0.5))


def _couple(l, r):
    """Forward square-polar coupling of quantised residues: (magnitude, angle)."""
    m = np.where(np.abs(l) > np.abs(r), l, r)
    a = np.where(np.abs(l) > np.abs(r), np.where(l > 0, l - r, r - l), np.where(r > 0, l - r, r - l))
    return m, a


def _uncouple(m, a):
    m, a = m.astype(F32), a.astype(F32)
    nm = np.where(m > 0, np.where(a > 0, m, m + a), np.where(a > 0, m, m - a)).astype(F32)
    na = np.where(m > 0, np.where(a > 0, m - a, m), np.where(a > 0, m + a, m)).astype(F32)
    return nm, na


def _residue_packet(w, rtype, qs, n2, psize):
    """Residues of the channels (int arrays of n2), classification per partition."""
    if rtype == 2:
        inter = np.stack(qs, axis=1).reshape(-1)
        vecs, size = [inter], n2 * len(qs)
    else:
        vecs, size = qs, n2
    parts = size // psize
    for p in range(parts):
        off = p * psize
        cls = [int(np.any(v[off:off + psize] != 0)) for v in vecs]
        for c in cls:
            BOOK_CLASS.emit(w, c)
        for v, c in zip(vecs, cls):
            if not c:
                continue
            seg = v[off:off + psize]
            if rtype == 0:
                step = psize // 2
                pairs = [(seg[j], seg[j + step]) for j in range(step)]
            else:
                pairs = [(seg[j], seg[j + 1]) for j in range(0, psize, 2)]
            for a, b in pairs:
                BOOK_VQ.emit(w, int(a) + 32 + VQ_VALUES * (int(b) + 32))


def headers(channels, rate, rtype, damage=None):
    """damage (malformed setup headers for the decoder's rejection paths): "mux" = two submaps
    with channel 0's mux equal to the submap count; "dup_x" = floor 0's X list repeats a value;
    "big_dims" = an extra lookup-type-2 book whose entries x dims is 2^32 (0 in 32 bits)."""
    idh = LBitWriter()
    idh.put(0, 32)
    idh.put(channels, 8)
    idh.put(rate, 32)
    for _ in range(3):
        idh.put(0, 32)
    idh.put(8, 4)   # blocksize 0 = 256
    idh.put(11, 4)  # blocksize 1 = 2048
    idh.put(1, 1)
    ident = b"\x01vorbis" + idh.bytes()
    cw = LBitWriter()
    vendor = b"stratum-hip test encoder"
    cw.put(len(vendor), 32)
    for ch in vendor:
        cw.put(ch, 8)
    cw.put(0, 32)
    cw.put(1, 1)
    comment = b"\x03vorbis" + cw.bytes()
    s = LBitWriter()
    s.put(len(BOOKS) - 1 + (damage == "big_dims"), 8)
    for b in BOOKS:
        b.write_header(s)
    if damage == "big_dims":  # 2^17 entries of 17 bits (a complete tree, ordered) x 32768 dimensions
        s.put(0x564342, 24)
        s.put(32768, 16)
        s.put(1 << 17, 24)
        s.put(1, 1)  # ordered: one run of 2^17 lengths of 17
        s.put(16, 5)
        s.put(1 << 17, 18)
        s.put(2, 4)
        s.put(float32_pack(0.0), 32)
        s.put(float32_pack(1.0), 32)
        s.put(0, 4)
        s.put(0, 1)
    s.put(0, 6)
    s.put(0, 16)
    s.put(len(FLOORS) - 1, 6)
    for i, f in enumerate(FLOORS):
        if damage == "dup_x" and i == 0:
            f = FloorSpec(f.rangebits, [f.X[2], f.X[2]] + f.X[4:])
        _write_floor(s, f)
    s.put(1, 6)  # 2 residues: short, long
    for n2, psize in [(128, 16), (1024, 32)]:
        s.put(rtype, 16)
        s.put(0, 24)
        s.put(n2 * (channels if rtype == 2 else 1), 24)
        s.put(psize - 1, 24)
        s.put(1, 6)   # 2 classifications
        s.put(1, 8)   # classbook BOOK_CLASS
        s.put(0, 3)   # class 0: no passes
        s.put(0, 1)
        s.put(1, 3)   # class 1: pass 0
        s.put(0, 1)
        s.put(2, 8)   # BOOK_VQ
    s.put(1, 6)  # 2 mappings
    for m in range(2):
        s.put(0, 16)
        s.put(int(damage == "mux"), 1)  # one submap (two with the "mux" damage)
        if damage == "mux":
            s.put(1, 4)
        if channels == 2:
            s.put(1, 1)
            s.put(0, 8)
            s.put(0, ilog(channels - 1))
            s.put(1, ilog(channels - 1))
        else:
            s.put(0, 1)
        s.put(0, 2)
        if damage == "mux":
            for c in range(channels):
                s.put(2 if c == 0 else 0, 4)  # channel 0 names submap 2 of {0, 1}
            s.put(0, 8)
            s.put(m, 8)
            s.put(m, 8)
        s.put(0, 8)
        s.put(m, 8)  # floor
        s.put(m, 8)  # residue
    s.put(1, 6)  # 2 modes
    for m in range(2):
        s.put(m, 1)
        s.put(0, 16)
        s.put(0, 16)
        s.put(m, 8)
    s.put(1, 1)
    setup = b"\x05vorbis" + s.bytes()
    return [ident, comment, setup]


def encode(chans, rate, pattern, rtype=1, silent_blocks=()):
    """chans: float arrays (one per channel); pattern: block flags (0 short, 1 long), one per
    block, the first block centred at sample 0.  Returns (packets, granules, expected), where
    expected is the float32 per-channel reconstruction of samples [0, total)."""
    C = len(chans)
    bs = [256, 2048]
    n_blocks = len(pattern)
    centres = [0]
    for k in range(1, n_blocks):
        centres.append(centres[-1] + bs[pattern[k - 1]] // 4 + bs[pattern[k]] // 4)
    total = centres[-1]
    pad = 4096
    xs = [np.concatenate([np.zeros(pad), np.asarray(c, np.float64), np.zeros(total + pad)]) for c in chans]
    packets, granules = [], []
    recon = [np.zeros(total + 2 * pad, np.float64) for _ in range(C)]
    outputs = [[] for _ in range(C)]
    prev = None
    for k in range(n_blocks):
        bf = pattern[k]
        n, n2 = bs[bf], bs[bf] // 2
        prev_long = bool(pattern[k - 1]) if k > 0 else True
        next_long = bool(pattern[k + 1]) if k + 1 < n_blocks else True
        win = window(n, bs[0], bf, prev_long, next_long)
        start = centres[k] - n // 2 + pad
        cm = _cos_matrix(n)
        spec = [4.0 / n * (cm.T @ (x[start:start + n] * win.astype(np.float64))) for x in xs]
        w = LBitWriter()
        w.put(0, 1)
        w.put(bf, 1)  # mode number (2 modes: 1 bit)
        if bf:
            w.put(int(prev_long), 1)
            w.put(int(next_long), 1)
        f = FLOORS[bf]
        silent = k in silent_blocks
        curves, qs = [], []
        for c in range(C):
            if silent and C == 1:
                w.put(0, 1)  # floor unused
                curves.append(None)
                qs.append(np.zeros(n2, np.int64))
                continue
            # targets: the floor index (0 .. 127, x 2) just above each region's peak / 12
            targets = []
            xs_sorted = sorted(f.X)
            for x in f.X:
                k = xs_sorted.index(x)  # the region between this point's neighbours
                lo = min(n2 - 1, xs_sorted[max(0, k - 1)])
                hi = max(lo + 1, min(n2, xs_sorted[min(len(xs_sorted) - 1, k + 1)] + 1))
                peak = max(np.max(np.abs(spec[c][lo:hi])), 1e-7) / 12.0
                idx = 255 - int(np.floor(-20.0 * np.log10(peak) / (140.0 / 256.0)))
                targets.append(min(127, max(1, (idx + 1) // 2)))
            Y = floor_values(f, targets)
            _write_floor_packet(w, Y)
            curve = floor_synthesis(f, Y, n2)
            curves.append(curve)
            lim = 16 if C == 2 else 32
            q = np.clip(np.round(spec[c] / curve.astype(np.float64)), -lim, lim).astype(np.int64)
            qs.append(q)
        if C == 2:
            m, a = _couple(qs[0], qs[1])
            coded = [m, a]
        else:
            coded = qs
        if not (silent and C == 1):
            _residue_packet(w, rtype, coded, n2, 16 if bf == 0 else 32)
        packets.append(w.bytes())
        # the decoder's reconstruction (float32 products, IMDCT by its sum, window, overlap-add)
        if C == 2:
            r0, r1 = _uncouple(coded[0], coded[1])
            res = [r0, r1]
        else:
            res = [q.astype(F32) for q in qs]
        cur = []
        for c in range(C):
            if curves[c] is None:
                s = np.zeros(n2, F32)
            else:
                s = (curves[c] * res[c]).astype(F32)
            y = (cm @ s.astype(np.float64)).astype(F32)
            cur.append((y * win).astype(F32))
        if prev is not None:
            pn = len(prev[0])
            L = pn // 4 + n // 4
            for c in range(C):
                seg = np.zeros(L, F32)
                for i in range(L):
                    pi, ci = pn // 2 + i, i - L + n // 2
                    pv = prev[c][pi] if pi < pn else F32(0)
                    cv = cur[c][ci] if ci >= 0 else F32(0)
                    seg[i] = F32(pv + cv)
                outputs[c].append(seg)
            granules.append(sum(len(s) for s in outputs[0]))
        else:
            granules.append(0)
        prev = cur
    expected = [np.concatenate(o) if o else np.zeros(0, F32) for o in outputs]
    return packets, granules, expected


def ogg_stream(headers_, packets, granules, final_len=None, serial=0x5EED):
    """One page per packet; headers at granule 0, audio pages at their cumulative output count
    (the last one cut to final_len when given)."""
    out = b""
    allp = [(h, 0) for h in headers_] + list(zip(packets, granules))
    for seq, (p, g) in enumerate(allp):
        if seq == len(allp) - 1 and final_len is not None:
            g = final_len
        segs = []
        i = 0
        while len(p) - i >= 255:
            segs.append(255)
            i += 255
        segs.append(len(p) - i)
        assert len(segs) <= 255
        flags = (2 if seq == 0 else 0) | (4 if seq == len(allp) - 1 else 0)
        hdr = b"OggS" + bytes([0, flags]) + struct.pack("<qIII", g, serial, seq, 0) + bytes([len(segs)]) + bytes(segs)
        page = bytearray(hdr + p)
        struct.pack_into("<I", page, 22, _crc(page))
        out += bytes(page)
    return out


def _crc(page):
    crc = 0
    for b in page:
        crc ^= b << 24
        for _ in range(8):
            crc = ((crc << 1) ^ 0x04C11DB7) if crc & 0x80000000 else (crc << 1)
            crc &= 0xFFFFFFFF
    return crc
