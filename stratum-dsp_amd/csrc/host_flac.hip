// host_flac.hip — native FLAC decoder for the decode front-end (sdsp_decode_audio_file).
//
// The reference decodes FLAC with symphonia 0.5 ("all" features, Cargo.toml:15) and converts each
// decoded buffer in its examples (examples/analyze_batch.rs:30-177, analyze_file.rs:25-180).
// symphonia's FLAC decoder delivers AudioBufferRef::S32 with every sample shifted left by
// 32 - bits_per_sample, which the examples turn into `s as f32 / 2147483648.0` (mono) or the
// channel sum from -0.0 divided by `channels as f32`.  Packets that fail to decode are skipped
// (`Err(DecodeError) => continue`), which this decoder mirrors per frame: a frame whose header
// CRC-8 or frame CRC-16 does not match, or whose subframes are malformed, is dropped and the
// scan resumes at the next frame sync code.  The sample rate is STREAMINFO's
// (codec_params.sample_rate, 44100 when absent).
//
// Format (FLAC, RFC 9639): "fLaC", metadata blocks (STREAMINFO first), then frames: a header
// (sync 0x3FFE, block size / sample rate / channel assignment / sample size codes, UTF-8 coded
// frame or sample number, CRC-8), one subframe per channel (CONSTANT, VERBATIM, FIXED order 0-4,
// LPC order 1-32; wasted bits; Rice or escaped residual partitions), zero padding to a byte and a
// CRC-16.  Stereo decorrelation: left/side, side/right, mid/side.  Decoding is integer-exact
// (64-bit prediction sums), so the f32 output depends only on the conversion above.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Bits {
    const uint8_t* p;
    size_t n, pos = 0;  // pos in bits
    bool bad = false;
    Bits(const uint8_t* d, size_t len) : p(d), n(len) {}
    uint64_t get(int k) {  // k <= 57
        uint64_t v = 0;
        for (int i = 0; i < k; i++) {
            if ((pos >> 3) >= n) {
                bad = true;
                return 0;
            }
            v = (v << 1) | ((p[pos >> 3] >> (7 - (pos & 7))) & 1u);
            pos++;
        }
        return v;
    }
    int64_t sget(int k) {  // two's complement, k <= 57
        if (k == 0) return 0;
        const uint64_t v = get(k);
        return (v >> (k - 1)) & 1u ? (int64_t)(v - (1ull << k)) : (int64_t)v;
    }
    uint64_t unary() {  // zeros before the terminating 1
        uint64_t q = 0;
        for (;;) {
            if ((pos >> 3) >= n) {
                bad = true;
                return 0;
            }
            const uint8_t byte = p[pos >> 3];
            const int off = (int)(pos & 7);
            const uint8_t rest = (uint8_t)(byte << off);
            if (rest == 0) {  // the rest of this byte is zeros
                q += (uint64_t)(8 - off);
                pos += (size_t)(8 - off);
                continue;
            }
            const int lz = __builtin_clz((unsigned)rest) - 24;
            q += (uint64_t)lz;
            pos += (size_t)lz + 1;
            return q;
        }
    }
    void align() { pos = (pos + 7) & ~(size_t)7; }
};

uint8_t crc8(const uint8_t* d, size_t n) {
    uint8_t c = 0;
    for (size_t i = 0; i < n; i++) {
        c ^= d[i];
        for (int b = 0; b < 8; b++) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : c << 1);
    }
    return c;
}
uint16_t crc16(const uint8_t* d, size_t n) {
    uint16_t c = 0;
    for (size_t i = 0; i < n; i++) {
        c ^= (uint16_t)(d[i] << 8);
        for (int b = 0; b < 8; b++) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x8005 : c << 1);
    }
    return c;
}

struct StreamInfo {
    uint32_t rate = 0;
    int channels = 0, bps = 0;
};

// residual of one subframe into r[order .. bs), false when malformed
bool residual(Bits& b, int order, uint32_t bs, int64_t* r) {
    const uint64_t method = b.get(2);
    if (method > 1) return false;
    const int pbits = method == 0 ? 4 : 5;
    const uint64_t esc = method == 0 ? 15 : 31;
    const int porder = (int)b.get(4);
    const uint32_t parts = 1u << porder;
    if ((bs >> porder) << porder != bs || (bs >> porder) < (uint32_t)order) return false;
    uint32_t i = (uint32_t)order;
    for (uint32_t pi = 0; pi < parts; pi++) {
        const uint32_t cnt = (bs >> porder) - (pi == 0 ? (uint32_t)order : 0u);
        const uint64_t k = b.get(pbits);
        if (k == esc) {
            const int nb = (int)b.get(5);
            for (uint32_t j = 0; j < cnt; j++) r[i++] = b.sget(nb);
        } else {
            for (uint32_t j = 0; j < cnt; j++) {
                const uint64_t q = b.unary();
                if (q > (1ull << 40)) return false;
                const uint64_t u = (q << k) | b.get((int)k);
                r[i++] = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
            }
        }
        if (b.bad) return false;
    }
    return true;
}

// one subframe of `bps` bits per sample into s[0 .. bs)
bool subframe(Bits& b, int bps, uint32_t bs, int64_t* s) {
    if (b.get(1) != 0) return false;
    const int type = (int)b.get(6);
    int wasted = 0;
    if (b.get(1)) wasted = (int)b.unary() + 1;
    if (b.bad || wasted >= bps) return false;
    const int w = bps - wasted;
    if (type == 0) {  // CONSTANT
        const int64_t v = b.sget(w);
        for (uint32_t i = 0; i < bs; i++) s[i] = v;
    } else if (type == 1) {  // VERBATIM
        for (uint32_t i = 0; i < bs; i++) s[i] = b.sget(w);
    } else if (type >= 8 && type <= 12) {  // FIXED
        const int order = type - 8;
        if ((uint32_t)order > bs) return false;
        for (int i = 0; i < order; i++) s[i] = b.sget(w);
        if (!residual(b, order, bs, s)) return false;
        for (uint32_t i = (uint32_t)order; i < bs; i++) {
            const int64_t r = s[i];
            switch (order) {
                case 0: s[i] = r; break;
                case 1: s[i] = r + s[i - 1]; break;
                case 2: s[i] = r + 2 * s[i - 1] - s[i - 2]; break;
                case 3: s[i] = r + 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
                default: s[i] = r + 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
            }
        }
    } else if (type >= 32) {  // LPC
        const int order = type - 31;
        if ((uint32_t)order > bs) return false;
        for (int i = 0; i < order; i++) s[i] = b.sget(w);
        const int prec = (int)b.get(4) + 1;
        if (prec == 16) return false;  // 0b1111 is invalid
        const int shift = (int)b.sget(5);
        if (shift < 0) return false;
        int64_t c[32];
        for (int j = 0; j < order; j++) c[j] = b.sget(prec);
        if (!residual(b, order, bs, s)) return false;
        for (uint32_t i = (uint32_t)order; i < bs; i++) {
            __int128 acc = 0;  // 32-bit coefficients times 33-bit samples, up to 32 terms
            for (int j = 0; j < order; j++) acc += (__int128)c[j] * s[i - 1 - j];
            s[i] += (int64_t)(acc >> shift);
        }
    } else {
        return false;  // reserved
    }
    if (b.bad) return false;
    if (wasted)
        for (uint32_t i = 0; i < bs; i++) s[i] = (int64_t)((uint64_t)s[i] << wasted);
    return true;
}

// frame header at f[pos]; returns its length in bytes (0: no valid header)
size_t frame_header(const uint8_t* f, size_t n, const StreamInfo& si, uint32_t* bs, int* bps, int* chan_code) {
    if (n < 6 || f[0] != 0xFF || (f[1] & 0xFE) != 0xF8) return 0;
    Bits b(f, n);
    b.get(16);
    const int bsc = (int)b.get(4), src = (int)b.get(4), chc = (int)b.get(4), ssc = (int)b.get(3);
    if (b.get(1) != 0 || bsc == 0 || src == 15 || chc > 10 || ssc == 3) return 0;
    // UTF-8 coded frame / sample number
    const uint64_t lead = b.get(8);
    int extra = 0;
    if (lead < 0x80) extra = 0;
    else if ((lead & 0xE0) == 0xC0) extra = 1;
    else if ((lead & 0xF0) == 0xE0) extra = 2;
    else if ((lead & 0xF8) == 0xF0) extra = 3;
    else if ((lead & 0xFC) == 0xF8) extra = 4;
    else if ((lead & 0xFE) == 0xFC) extra = 5;
    else if (lead == 0xFE) extra = 6;
    else return 0;
    for (int i = 0; i < extra; i++)
        if ((b.get(8) & 0xC0) != 0x80) return 0;
    static const uint32_t fixed_bs[16] = {0, 192, 576, 1152, 2304, 4608, 0, 0, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768};
    if (bsc == 6) *bs = (uint32_t)b.get(8) + 1;
    else if (bsc == 7) *bs = (uint32_t)b.get(16) + 1;
    else *bs = fixed_bs[bsc];
    if (src == 12) b.get(8);
    else if (src == 13 || src == 14) b.get(16);
    if (b.bad) return 0;
    const size_t hl = b.pos / 8;
    if (hl + 1 > n || crc8(f, hl) != f[hl]) return 0;
    static const int fixed_bps[8] = {0, 8, 12, 0, 16, 20, 24, 32};
    *bps = ssc == 0 ? si.bps : fixed_bps[ssc];
    *chan_code = chc;
    return hl + 1;
}

}  // namespace

// Decodes a FLAC stream (f) into mono f32 (the reference examples' conversion) and its rate.
bool sdsp_decode_flac(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err) {
    size_t pos = 0;
    if (f.size() >= 10 && std::memcmp(f.data(), "ID3", 3) == 0) {  // an ID3v2 tag ahead of the stream
        const size_t sz = ((size_t)(f[6] & 0x7F) << 21) | ((size_t)(f[7] & 0x7F) << 14) | ((size_t)(f[8] & 0x7F) << 7) |
                          (size_t)(f[9] & 0x7F);
        pos = 10 + sz + ((f[5] & 0x10) ? 10 : 0);
    }
    if (f.size() < pos + 4 || std::memcmp(f.data() + pos, "fLaC", 4) != 0) {
        *err = "not a FLAC stream";
        return false;
    }
    pos += 4;
    StreamInfo si;
    bool have_si = false, last = false;
    while (!last) {
        if (pos + 4 > f.size()) {
            *err = "truncated FLAC metadata";
            return false;
        }
        last = (f[pos] & 0x80) != 0;
        const int type = f[pos] & 0x7F;
        const size_t len = ((size_t)f[pos + 1] << 16) | ((size_t)f[pos + 2] << 8) | f[pos + 3];
        pos += 4;
        if (pos + len > f.size()) {
            *err = "truncated FLAC metadata block";
            return false;
        }
        if (type == 0) {
            if (len < 34) {
                *err = "malformed STREAMINFO";
                return false;
            }
            Bits b(f.data() + pos, len);
            b.get(16);  // min block size
            b.get(16);  // max block size
            b.get(24);  // min frame size
            b.get(24);  // max frame size
            si.rate = (uint32_t)b.get(20);
            si.channels = (int)b.get(3) + 1;
            si.bps = (int)b.get(5) + 1;
            have_si = true;
        }
        pos += len;
    }
    if (!have_si) {
        *err = "missing STREAMINFO";
        return false;
    }
    if (si.bps < 4 || si.bps > 32) {
        *err = "unsupported FLAC bits per sample " + std::to_string(si.bps);
        return false;
    }
    std::vector<int64_t> ch[8];
    out->clear();
    const uint8_t* d = f.data();
    const size_t n = f.size();
    while (pos + 2 <= n) {
        uint32_t bs = 0;
        int bps = 0, chc = 0;
        const size_t hl = frame_header(d + pos, n - pos, si, &bs, &bps, &chc);
        if (hl == 0) {  // not a frame start: resynchronise one byte later
            pos++;
            continue;
        }
        const int nch = chc <= 7 ? chc + 1 : 2;
        bool ok = bps >= 4 && bps <= 32 && bs > 0;
        Bits b(d + pos + hl, n - pos - hl);
        for (int c = 0; ok && c < nch; c++) {
            ch[c].assign(bs, 0);
            const bool side = (chc == 8 && c == 1) || (chc == 9 && c == 0) || (chc == 10 && c == 1);
            ok = subframe(b, bps + (side ? 1 : 0), bs, ch[c].data());
        }
        size_t end = 0;
        if (ok) {
            b.align();
            end = pos + hl + b.pos / 8;
            ok = end + 2 <= n && crc16(d + pos, end - pos) == (uint16_t)((d[end] << 8) | d[end + 1]);
        }
        if (!ok) {  // DecodeError: the packet is skipped (analyze_batch.rs `continue`)
            pos++;
            continue;
        }
        if (chc == 8) {
            for (uint32_t i = 0; i < bs; i++) ch[1][i] = ch[0][i] - ch[1][i];  // left, side -> right
        } else if (chc == 9) {
            for (uint32_t i = 0; i < bs; i++) ch[0][i] = ch[0][i] + ch[1][i];  // side, right -> left
        } else if (chc == 10) {
            for (uint32_t i = 0; i < bs; i++) {
                const int64_t side = ch[1][i];
                const int64_t mid = (int64_t)((uint64_t)ch[0][i] << 1) | (side & 1);
                ch[0][i] = (mid + side) >> 1;
                ch[1][i] = (mid - side) >> 1;
            }
        }
        // symphonia's S32 buffer: sample << (32 - bps); the examples' S32 conversion
        const int shift = 32 - bps;
        auto conv = [&](int64_t v) {
            const int32_t s32 = (int32_t)(uint32_t)((uint64_t)v << shift);
            return (float)s32 / 2147483648.0f;
        };
        const size_t o = out->size();
        out->resize(o + bs);
        for (uint32_t i = 0; i < bs; i++) {
            if (nch == 1) {
                (*out)[o + i] = conv(ch[0][i]);
            } else {
                float s = -0.0f;
                for (int c = 0; c < nch; c++) s = s + conv(ch[c][i]);
                (*out)[o + i] = s / (float)nch;
            }
        }
        pos = end + 2;
    }
    *sr = si.rate ? si.rate : 44100u;
    return true;
}
