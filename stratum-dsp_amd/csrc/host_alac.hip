// host_alac.hip — Apple Lossless (ALAC) in CAF and ISO MP4 (.m4a) for the decode front-end.
//
// The reference decodes ALAC through symphonia's ALAC codec and CAF / ISO MP4 readers
// (Cargo.toml:15, features = ["all"]); the examples convert the decoded buffer to mono f32
// (examples/analyze_file.rs:25-180).  ALAC is lossless, so a decoder's output is the encoded
// PCM whatever its internals; this one follows Apple's published ALAC format (ALACSpecificConfig
// magic cookie; per frame the SCE / CPE elements, each compressed with the adaptive Golomb coder
// and the sign-adaptive FIR predictor, or escaped as raw samples; "bytes shifted" low bits; the
// stereo un-mixing; the END tag).  Samples reach the examples' conversion as integers of the
// stream's bit depth: 16 -> s / 32768, 20 and 24 -> s / 2^(bits-1) (S24 / S32 buffers give the
// same f32 values for these depths), 32 -> s / 2^31.  One and two channels (SCE, CPE) are
// decoded; other channel layouts are a decoding error.  Parity with symphonia itself is
// unpinned: tests/alac_enc.py writes the test streams from the same format description.
#include <cstring>
#include <string>
#include <vector>

namespace {

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }

bool fail(std::string* err, const std::string& m) {
    *err = m;
    return false;
}

struct AlacConfig {
    uint32_t frame_length = 4096;
    int bit_depth = 16, pb = 40, mb = 10, kb = 14, channels = 2, max_run = 255;
    uint32_t sample_rate = 44100;
};

// ALACSpecificConfig (24 bytes), possibly behind 'frma' / 'alac' atom headers (CAF 'kuki')
bool parse_cookie(const uint8_t* p, size_t n, AlacConfig* c, std::string* err) {
    if (n >= 12 && std::memcmp(p + 4, "frma", 4) == 0) p += 12, n -= 12;
    if (n >= 12 && std::memcmp(p + 4, "alac", 4) == 0) p += 12, n -= 12;
    if (n < 24) return fail(err, "malformed ALAC magic cookie");
    c->frame_length = be32(p);
    c->bit_depth = p[5];
    c->pb = p[6];
    c->mb = p[7];
    c->kb = p[8];
    c->channels = p[9];
    c->max_run = be16(p + 10);
    c->sample_rate = be32(p + 20);
    if (c->frame_length == 0 || c->frame_length > (1u << 20)) return fail(err, "unsupported ALAC frame length");
    if (c->bit_depth != 16 && c->bit_depth != 20 && c->bit_depth != 24 && c->bit_depth != 32)
        return fail(err, "unsupported ALAC bit depth " + std::to_string(c->bit_depth));
    if (c->channels < 1 || c->channels > 2) return fail(err, "unsupported ALAC channel count " + std::to_string(c->channels));
    if (c->kb < 1 || c->kb > 14) return fail(err, "malformed ALAC magic cookie");
    return true;
}

// MSB-first bit reader over one packet; reads past the end return zeros and set `over`
struct Bits {
    const uint8_t* p;
    size_t n;
    uint64_t pos = 0;
    bool over = false;
    Bits(const uint8_t* d, size_t len) : p(d), n(len) {}
    uint32_t peek32() const {  // the 32 bits at pos (zeros past the end)
        uint64_t w = 0;
        for (int i = 0; i < 5; i++) {
            const size_t b = (size_t)(pos >> 3) + (size_t)i;
            w = (w << 8) | (b < n ? p[b] : 0);
        }
        return (uint32_t)(w >> (8 - (pos & 7)));
    }
    uint32_t read(int k) {  // k <= 32
        if (k == 0) return 0;
        const uint32_t v = k == 32 ? peek32() : peek32() >> (32 - k);
        pos += (uint64_t)k;
        if (pos > 8 * (uint64_t)n) over = true;
        return v;
    }
    void skip(uint64_t k) {
        pos += k;
        if (pos > 8 * (uint64_t)n) over = true;
    }
};

inline int clz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }

// adaptive Golomb parameters (Apple's ag_dec: QBSHIFT 9, MMULSHIFT 2, MDENSHIFT 6, MOFF 16,
// BITOFF 24, escape after a 9-bit prefix, zero runs of up to 65535)
constexpr int QBSHIFT = 9, QB = 1 << QBSHIFT, MMULSHIFT = 2, MDENSHIFT = QBSHIFT - MMULSHIFT - 1,
              MOFF = 1 << (MDENSHIFT - 2), BITOFF = 24, MAX_PREFIX = 9, MAX_DATATYPE_BITS_16 = 16;

// one Golomb value: a unary prefix of ones (escape at 9), then k bits; values v < 2 give pre * m
// and return the k-th bit to the stream
uint32_t ag_get(Bits& b, uint32_t m, int k, int escape_bits) {
    const uint32_t s = b.peek32();
    const int pre = clz32(~s);
    if (pre >= MAX_PREFIX) {
        b.skip(MAX_PREFIX);
        return b.read(escape_bits);
    }
    b.skip((uint64_t)pre + 1);
    if (k == 1) return (uint32_t)pre;
    const uint32_t v = b.read(k);
    if (v >= 2) return (uint32_t)pre * m + v - 1;
    b.pos -= 1;
    return (uint32_t)pre * m;
}

// dyn_decomp: numSamples signed residuals into pc
bool ag_decode(Bits& b, const AlacConfig& c, int pb_factor, int n, int chan_bits, std::vector<int32_t>& pc) {
    const uint32_t pb = (uint32_t)(c.pb * pb_factor) / 4;
    const uint32_t wb = (1u << c.kb) - 1;
    uint32_t mb = (uint32_t)c.mb;
    uint32_t zmode = 0;
    int i = 0;
    while (i < n) {
        const uint32_t m0 = mb >> QBSHIFT;
        int k = 31 - clz32(m0 + 3);  // lg3a
        if (k > c.kb) k = c.kb;
        const uint32_t m = (1u << k) - 1;
        const uint32_t v = ag_get(b, m, k, chan_bits);
        const uint32_t nd = v + zmode;
        const int32_t mag = (int32_t)((nd + 1) >> 1);
        pc[(size_t)i++] = (nd & 1) ? -mag : mag;
        mb = pb * (v + zmode) + mb - ((pb * mb) >> QBSHIFT);
        if (v > 0xffff) mb = 0xffff;
        zmode = 0;
        if (((mb << MMULSHIFT) < (uint32_t)QB) && i < n) {
            zmode = 1;
            const int kz = clz32(mb) - BITOFF + (int)((mb + MOFF) >> MDENSHIFT);
            const uint32_t mz = ((1u << kz) - 1) & wb;
            const uint32_t run = ag_get(b, mz, kz, MAX_DATATYPE_BITS_16);
            if ((uint64_t)i + run > (uint64_t)n) return false;
            for (uint32_t j = 0; j < run; j++) pc[(size_t)i++] = 0;
            if (run >= 65535) zmode = 0;
            mb = 0;
        }
        if (b.over) return false;
    }
    return true;
}

inline int32_t sext(int32_t v, int chan_bits) {
    const int sh = 32 - chan_bits;
    return (int32_t)((uint32_t)v << sh) >> sh;
}
inline int32_t sign_of(int32_t v) { return (v > 0) - (v < 0); }

// unpc_block: the sign-adaptive predictor (numactive 31: first-order difference)
void unpredict(const std::vector<int32_t>& pc, std::vector<int32_t>& out, int n, int16_t* coefs, int na, int chan_bits,
               int den_shift) {
    if (n <= 0) return;
    out[0] = pc[0];
    if (na == 0) {
        for (int j = 1; j < n; j++) out[(size_t)j] = pc[(size_t)j];
        return;
    }
    if (na == 31) {
        int32_t prev = out[0];
        for (int j = 1; j < n; j++) {
            prev = sext((int32_t)((uint32_t)pc[(size_t)j] + (uint32_t)prev), chan_bits);
            out[(size_t)j] = prev;
        }
        return;
    }
    for (int j = 1; j <= na && j < n; j++)
        out[(size_t)j] = sext((int32_t)((uint32_t)pc[(size_t)j] + (uint32_t)out[(size_t)j - 1]), chan_bits);
    const int32_t den_half = den_shift > 0 ? 1 << (den_shift - 1) : 0;
    const int lim = na + 1;
    for (int j = lim; j < n; j++) {
        const int32_t* pout = out.data() + j - 1;
        const int32_t top = out[(size_t)(j - lim)];
        // 32-bit wrap-around arithmetic, as the reference implementation's int32 sums
        uint32_t sum = 0;
        for (int k = 0; k < na; k++) sum += (uint32_t)((int64_t)coefs[k] * ((int64_t)pout[-k] - (int64_t)top));
        const int32_t del = pc[(size_t)j];
        int32_t del0 = del;
        const int32_t sg = sign_of(del);
        const int32_t pred = (int32_t)(sum + (uint32_t)den_half) >> den_shift;
        out[(size_t)j] = sext((int32_t)((uint32_t)del + (uint32_t)top + (uint32_t)pred), chan_bits);
        if (sg > 0) {
            for (int k = na - 1; k >= 0; k--) {
                const int32_t dd = (int32_t)((uint32_t)top - (uint32_t)pout[-k]);
                const int32_t sgn = sign_of(dd);
                coefs[k] = (int16_t)(coefs[k] - sgn);
                del0 -= (na - k) * (int32_t)((int64_t)sgn * dd >> den_shift);
                if (del0 <= 0) break;
            }
        } else if (sg < 0) {
            for (int k = na - 1; k >= 0; k--) {
                const int32_t dd = (int32_t)((uint32_t)top - (uint32_t)pout[-k]);
                const int32_t sgn = sign_of(dd);
                coefs[k] = (int16_t)(coefs[k] + sgn);
                del0 -= (na - k) * (int32_t)((int64_t)-sgn * dd >> den_shift);
                if (del0 >= 0) break;
            }
        }
    }
}

// one ALAC frame (packet) -> interleaved integer samples appended to pcm
bool decode_frame(const uint8_t* d, size_t len, const AlacConfig& c, std::vector<int32_t>* pcm, std::string* err) {
    Bits b(d, len);
    const int nch_total = c.channels;
    int ch_done = 0;
    std::vector<int32_t> frame_out;
    int frame_n = -1;
    while (true) {
        const uint32_t tag = b.read(3);
        if (b.over) return fail(err, "truncated ALAC frame");
        if (tag == 7) break;  // ID_END
        if (tag == 6) {       // ID_FIL: count + bytes
            uint32_t cnt = b.read(4);
            if (cnt == 15) cnt += b.read(8) - 1;
            b.skip(8ull * cnt);
            continue;
        }
        if (tag == 4) {  // ID_DSE: tag, align flag, count, (align), bytes
            b.read(4);
            const uint32_t align = b.read(1);
            uint32_t cnt = b.read(8);
            if (cnt == 255) cnt += b.read(8);
            if (align) b.skip((8 - (b.pos & 7)) & 7);
            b.skip(8ull * cnt);
            continue;
        }
        if (tag != 0 && tag != 1 && tag != 3) return fail(err, "unsupported ALAC element " + std::to_string(tag));
        const int ech = tag == 1 ? 2 : 1;
        if (ch_done + ech > nch_total) return fail(err, "ALAC element exceeds the channel count");
        b.read(4);  // element instance tag
        if (b.read(12) != 0) return fail(err, "malformed ALAC element header");
        const uint32_t hb = b.read(4);
        const bool partial = hb & 8;
        const int bytes_shifted = (int)((hb >> 1) & 3);
        const bool escape = hb & 1;
        if (bytes_shifted == 3) return fail(err, "malformed ALAC element header");
        int n = (int)c.frame_length;
        if (partial) {
            uint32_t v = b.read(16) << 16;
            v |= b.read(16);
            if (v == 0 || v > c.frame_length) return fail(err, "malformed ALAC sample count");
            n = (int)v;
        }
        if (frame_n < 0) {
            frame_n = n;
            frame_out.assign((size_t)n * (size_t)nch_total, 0);
        } else if (n != frame_n) {
            return fail(err, "ALAC elements disagree on the sample count");
        }
        const int shift = escape ? 0 : bytes_shifted * 8;  // raw elements carry the full samples
        std::vector<int32_t> u((size_t)n), v(ech == 2 ? (size_t)n : 0), sh((size_t)n * (size_t)ech, 0);
        int mix_bits = 0, mix_res = 0;
        if (!escape) {
            const int chan_bits = c.bit_depth - shift + (ech == 2 ? 1 : 0);
            if (chan_bits < 1 || chan_bits > 32) return fail(err, "malformed ALAC element");
            if (ech == 2) {
                mix_bits = (int)b.read(8);
                mix_res = (int8_t)b.read(8);
                if (mix_bits > 31) return fail(err, "malformed ALAC element");
            }
            int mode[2], den[2], pbf[2], na[2];
            int16_t coefs[2][32];
            for (int e = 0; e < ech; e++) {
                const uint32_t h1 = b.read(8), h2 = b.read(8);
                mode[e] = (int)(h1 >> 4);
                den[e] = (int)(h1 & 15);
                pbf[e] = (int)(h2 >> 5);
                na[e] = (int)(h2 & 31);
                for (int k = 0; k < na[e]; k++) coefs[e][k] = (int16_t)b.read(16);
            }
            uint64_t shift_pos = 0;
            if (shift) {
                shift_pos = b.pos;
                b.skip((uint64_t)shift * (uint64_t)ech * (uint64_t)n);
            }
            std::vector<int32_t> pc((size_t)n);
            for (int e = 0; e < ech; e++) {
                if (!ag_decode(b, c, pbf[e], n, chan_bits, pc)) return fail(err, "corrupt ALAC residuals");
                std::vector<int32_t>& dst = e == 0 ? u : v;
                if (mode[e] == 0) {
                    unpredict(pc, dst, n, coefs[e], na[e], chan_bits, den[e]);
                } else if (mode[e] == 15) {  // a first-order pass, then the FIR predictor
                    std::vector<int32_t> tmp((size_t)n);
                    unpredict(pc, tmp, n, nullptr, 31, chan_bits, 0);
                    unpredict(tmp, dst, n, coefs[e], na[e], chan_bits, den[e]);
                } else {
                    return fail(err, "unsupported ALAC prediction mode " + std::to_string(mode[e]));
                }
            }
            if (shift) {
                const uint64_t end = b.pos;
                b.pos = shift_pos;
                for (int i = 0; i < n; i++)
                    for (int e = 0; e < ech; e++) sh[(size_t)i * ech + e] = (int32_t)b.read(shift);
                b.pos = end;
            }
        } else {
            // escaped: raw samples of the full bit depth, channels interleaved per sample
            const int bits = c.bit_depth;
            for (int i = 0; i < n; i++) {
                for (int e = 0; e < ech; e++) {
                    int32_t val;
                    if (bits <= 16) {
                        val = sext((int32_t)b.read(bits), bits);
                    } else {
                        const int32_t hi = sext((int32_t)b.read(16), 16);
                        val = (int32_t)((uint32_t)hi << (bits - 16)) | (int32_t)b.read(bits - 16);
                    }
                    (e == 0 ? u : v)[(size_t)i] = val;
                }
            }
        }
        if (b.over) return fail(err, "truncated ALAC frame");
        // un-mix (stereo) and restore the shifted low bytes
        for (int i = 0; i < n; i++) {
            int32_t l, r = 0;
            if (ech == 2) {
                if (mix_res != 0) {
                    l = (int32_t)((uint32_t)u[(size_t)i] + (uint32_t)v[(size_t)i] -
                                  (uint32_t)((int32_t)((uint32_t)mix_res * (uint32_t)v[(size_t)i]) >> mix_bits));
                    r = (int32_t)((uint32_t)l - (uint32_t)v[(size_t)i]);
                } else {
                    l = u[(size_t)i];
                    r = v[(size_t)i];
                }
            } else {
                l = u[(size_t)i];
            }
            if (shift) {
                l = (int32_t)((uint32_t)l << shift) | sh[(size_t)i * ech];
                if (ech == 2) r = (int32_t)((uint32_t)r << shift) | sh[(size_t)i * ech + 1];
            }
            frame_out[(size_t)i * nch_total + ch_done] = l;
            if (ech == 2) frame_out[(size_t)i * nch_total + ch_done + 1] = r;
        }
        ch_done += ech;
    }
    if (ch_done != nch_total) return fail(err, "ALAC frame is missing channels");
    pcm->insert(pcm->end(), frame_out.begin(), frame_out.end());
    return true;
}

// interleaved integers of the stream's depth -> mono f32 (the examples' conversion)
void to_mono(const AlacConfig& c, const std::vector<int32_t>& pcm, std::vector<float>* out) {
    const int ch = c.channels;
    const float scale = c.bit_depth == 16 ? 32768.0f : c.bit_depth == 32 ? 2147483648.0f : (float)(1u << (c.bit_depth - 1));
    const size_t frames = pcm.size() / (size_t)ch;
    out->resize(frames);
    for (size_t i = 0; i < frames; i++) {
        if (ch == 1) {
            (*out)[i] = (float)pcm[i] / scale;
        } else {
            float s = -0.0f;
            for (int k = 0; k < ch; k++) s = s + (float)pcm[i * ch + (size_t)k] / scale;
            (*out)[i] = s / (float)ch;
        }
    }
}

// packets -> mono; a packet that fails to decode is skipped (the examples skip DecodeError)
bool decode_packets(const AlacConfig& c, const uint8_t* base, size_t size, const std::vector<std::pair<uint64_t, uint64_t>>& pk,
                    std::vector<float>* out, uint32_t* sr, std::string* err) {
    std::vector<int32_t> pcm;
    for (const auto& p : pk) {
        if (p.first > size || p.second > size - p.first) return fail(err, "ALAC packet outside the file");
        std::string why;
        std::vector<int32_t> one;
        if (decode_frame(base + p.first, (size_t)p.second, c, &one, &why)) pcm.insert(pcm.end(), one.begin(), one.end());
    }
    to_mono(c, pcm, out);
    *sr = c.sample_rate ? c.sample_rate : 44100u;
    return true;
}

// CAF variable-length integer (pakt table)
bool caf_vlq(const uint8_t* p, size_t n, size_t* pos, uint64_t* v) {
    *v = 0;
    for (int i = 0; i < 10; i++) {
        if (*pos >= n) return false;
        const uint8_t b = p[(*pos)++];
        *v = (*v << 7) | (b & 0x7f);
        if (!(b & 0x80)) return true;
    }
    return false;
}

}  // namespace

// CAF with format 'alac': desc, kuki (the magic cookie), pakt (packet sizes), data
bool sdsp_decode_caf_alac(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err) {
    AlacConfig c;
    bool have_cookie = false;
    const uint8_t* pakt = nullptr;
    uint64_t pakt_len = 0;
    uint64_t data_off = 0, data_len = 0;
    bool have_data = false;
    size_t pos = 8;
    while (pos + 12 <= f.size()) {
        const uint8_t* ck = f.data() + pos;
        const int64_t slen = (int64_t)be64(ck + 4);
        const uint64_t avail = f.size() - (pos + 12);
        const uint64_t body = (slen < 0 || (uint64_t)slen > avail) ? avail : (uint64_t)slen;
        if (std::memcmp(ck, "kuki", 4) == 0) {
            if (!parse_cookie(ck + 12, (size_t)body, &c, err)) return false;
            have_cookie = true;
        } else if (std::memcmp(ck, "pakt", 4) == 0) {
            pakt = ck + 12;
            pakt_len = body;
        } else if (std::memcmp(ck, "data", 4) == 0) {
            if (body < 4) return fail(err, "malformed data chunk");
            data_off = pos + 16;
            data_len = body - 4;
            have_data = true;
        }
        if (slen < 0) break;
        pos += 12 + (uint64_t)slen;
    }
    if (!have_cookie) return fail(err, "missing ALAC magic cookie");
    if (!have_data) return fail(err, "missing data chunk");
    if (!pakt || pakt_len < 24) return fail(err, "missing packet table");
    const uint64_t npk = be64(pakt);
    std::vector<std::pair<uint64_t, uint64_t>> pk;
    size_t q = 24;
    uint64_t off = data_off;
    for (uint64_t i = 0; i < npk; i++) {
        uint64_t sz;
        if (!caf_vlq(pakt, (size_t)pakt_len, &q, &sz)) return fail(err, "malformed packet table");
        if (off + sz > data_off + data_len) return fail(err, "packet table exceeds the data chunk");
        pk.push_back({off, sz});
        off += sz;
    }
    return decode_packets(c, f.data(), f.size(), pk, out, sr, err);
}

namespace {
// ISO BMFF box walk: calls fn(type, body, body_len) for each box in [p, p + n)
template <class Fn>
bool boxes(const uint8_t* p, uint64_t n, Fn fn) {
    uint64_t pos = 0;
    while (pos + 8 <= n) {
        uint64_t sz = be32(p + pos);
        uint64_t hdr = 8;
        if (sz == 1) {
            if (pos + 16 > n) return false;
            sz = be64(p + pos + 8);
            hdr = 16;
        } else if (sz == 0) {
            sz = n - pos;
        }
        if (sz < hdr || pos + sz > n) return false;
        if (!fn(p + pos + 4, p + pos + hdr, sz - hdr)) return false;
        pos += sz;
    }
    return true;
}
}  // namespace

// ISO MP4 / M4A: the first audio track's sample table (stsd 'alac', stsz, stsc, stco / co64)
bool sdsp_decode_mp4(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err) {
    const uint8_t* moov = nullptr;
    uint64_t moov_n = 0;
    boxes(f.data(), f.size(), [&](const uint8_t* t, const uint8_t* b, uint64_t n) {
        if (std::memcmp(t, "moov", 4) == 0) moov = b, moov_n = n;
        return true;
    });
    if (!moov) return fail(err, "malformed ISO MP4 file: missing moov box");
    std::string codec;
    bool found = false;
    AlacConfig c;
    std::vector<uint32_t> sizes;
    std::vector<uint64_t> chunk_off;
    std::vector<uint32_t> stsc;  // triples: first chunk, samples per chunk, description index
    std::string why;
    boxes(moov, moov_n, [&](const uint8_t* t, const uint8_t* b, uint64_t n) {
        if (found || std::memcmp(t, "trak", 4) != 0) return true;
        const uint8_t* mdia = nullptr;
        uint64_t mdia_n = 0;
        boxes(b, n, [&](const uint8_t* t2, const uint8_t* b2, uint64_t n2) {
            if (std::memcmp(t2, "mdia", 4) == 0) mdia = b2, mdia_n = n2;
            return true;
        });
        if (!mdia) return true;
        bool audio = false;
        const uint8_t* stbl = nullptr;
        uint64_t stbl_n = 0;
        boxes(mdia, mdia_n, [&](const uint8_t* t3, const uint8_t* b3, uint64_t n3) {
            if (std::memcmp(t3, "hdlr", 4) == 0 && n3 >= 12 && std::memcmp(b3 + 8, "soun", 4) == 0) audio = true;
            if (std::memcmp(t3, "minf", 4) == 0)
                boxes(b3, n3, [&](const uint8_t* t4, const uint8_t* b4, uint64_t n4) {
                    if (std::memcmp(t4, "stbl", 4) == 0) stbl = b4, stbl_n = n4;
                    return true;
                });
            return true;
        });
        if (!audio || !stbl) return true;
        found = true;
        boxes(stbl, stbl_n, [&](const uint8_t* t5, const uint8_t* b5, uint64_t n5) {
            if (std::memcmp(t5, "stsd", 4) == 0 && n5 >= 16) {
                // first sample entry: size, format, 6 reserved + data ref index, then the audio
                // sample entry (20 bytes) and its child boxes
                const uint8_t* e = b5 + 8;
                const uint64_t esz = be32(e);
                codec.assign((const char*)e + 4, 4);
                if (codec == "alac" && esz >= 36 && 8 + esz <= n5)
                    boxes(e + 36, esz - 36, [&](const uint8_t* t6, const uint8_t* b6, uint64_t n6) {
                        if (std::memcmp(t6, "alac", 4) == 0 && n6 >= 28)
                            if (!parse_cookie(b6 + 4, (size_t)n6 - 4, &c, &why)) codec = "bad";
                        return true;
                    });
            } else if (std::memcmp(t5, "stsz", 4) == 0 && n5 >= 12) {
                const uint32_t fixed = be32(b5 + 4), cnt = be32(b5 + 8);
                if (fixed)
                    sizes.assign(cnt, fixed);
                else
                    for (uint32_t i = 0; i < cnt && 12 + 4 * (uint64_t)i + 4 <= n5; i++) sizes.push_back(be32(b5 + 12 + 4 * i));
            } else if (std::memcmp(t5, "stco", 4) == 0 && n5 >= 8) {
                const uint32_t cnt = be32(b5 + 4);
                for (uint32_t i = 0; i < cnt && 8 + 4 * (uint64_t)i + 4 <= n5; i++) chunk_off.push_back(be32(b5 + 8 + 4 * i));
            } else if (std::memcmp(t5, "co64", 4) == 0 && n5 >= 8) {
                const uint32_t cnt = be32(b5 + 4);
                for (uint32_t i = 0; i < cnt && 8 + 8 * (uint64_t)i + 8 <= n5; i++) chunk_off.push_back(be64(b5 + 8 + 8 * i));
            } else if (std::memcmp(t5, "stsc", 4) == 0 && n5 >= 8) {
                const uint32_t cnt = be32(b5 + 4);
                for (uint32_t i = 0; i < cnt && 8 + 12 * (uint64_t)i + 12 <= n5; i++)
                    for (int k = 0; k < 3; k++) stsc.push_back(be32(b5 + 8 + 12 * i + 4 * k));
            }
            return true;
        });
        return true;
    });
    if (!found) return fail(err, "ISO MP4 file without an audio track");
    if (codec == "bad") return fail(err, why);
    if (codec == "mp4a") return fail(err, "unsupported codec: AAC (ISO MP4)");
    if (codec != "alac") return fail(err, "unsupported codec: ISO MP4 '" + codec + "'");
    if (stsc.empty() || chunk_off.empty()) return fail(err, "malformed sample table");
    // sample -> (offset, size) through the sample-to-chunk runs
    std::vector<std::pair<uint64_t, uint64_t>> pk;
    size_t s = 0;
    const size_t runs = stsc.size() / 3;
    for (size_t r = 0; r < runs && s < sizes.size(); r++) {
        const uint64_t first = stsc[3 * r], per = stsc[3 * r + 1];
        const uint64_t last = r + 1 < runs ? stsc[3 * (r + 1)] : (uint64_t)chunk_off.size() + 1;
        if (first < 1 || last < first) return fail(err, "malformed sample table");
        for (uint64_t ch = first; ch < last && ch <= chunk_off.size() && s < sizes.size(); ch++) {
            uint64_t off = chunk_off[(size_t)ch - 1];
            for (uint64_t k = 0; k < per && s < sizes.size(); k++, s++) {
                pk.push_back({off, sizes[s]});
                off += sizes[s];
            }
        }
    }
    return decode_packets(c, f.data(), f.size(), pk, out, sr, err);
}

// ALAC from a magic cookie and a list of packets (the Matroska A_ALAC track, host_mkv.hip)
bool sdsp_decode_alac_packets(const std::vector<uint8_t>& cookie, const std::vector<std::vector<uint8_t>>& packets,
                              std::vector<float>* out, uint32_t* sr, std::string* err) {
    AlacConfig c;
    if (!parse_cookie(cookie.data(), cookie.size(), &c, err)) return false;
    std::vector<uint8_t> flat;
    std::vector<std::pair<uint64_t, uint64_t>> pk;
    for (const auto& p : packets) {
        pk.push_back({flat.size(), p.size()});
        flat.insert(flat.end(), p.begin(), p.end());
    }
    return decode_packets(c, flat.data(), flat.size(), pk, out, sr, err);
}
