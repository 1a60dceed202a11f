// host_formats.hip — the decode front-end's other containers (sdsp_decode_audio_file dispatches
// here by magic number; RIFF/WAVE and native FLAC are host_decode.hip / host_flac.hip).
//
// The reference decodes with symphonia 0.5 built with every feature (Cargo.toml:15) and turns each
// decoded buffer into mono f32 by its type (examples/analyze_file.rs:25-180, analyze_batch.rs:
// 30-177): F32 as is, F64 `as f32`, S16 / 32768, S24 / 8388608, S32 / 2147483648, U8 (s - 128) /
// 128, several channels summed in channel order (from -0.0) then divided by the channel count;
// any other buffer type (S8, U16, ...) is the examples' "Unsupported audio format" error.  The
// containers and codecs here decode to those buffer types as symphonia's readers do:
//   AIFF / AIFF-C   big-endian PCM ('NONE', 'twos': 16 / 24 / 32 bits -> S16 / S24 / S32; 8 bits is
//                   signed -> S8, unsupported), 'sowt' little-endian PCM, 'fl32' / 'fl64' floats,
//                   G.711 'alaw' / 'ulaw' (-> S16); the sample rate from the 80-bit extended float;
//   CAF             'lpcm' (integer: signed, big- or little-endian by the format flags; floats),
//                   'alaw' / 'ulaw', 'alac' (host_alac.hip);
//   Ogg             the FLAC mapping (first packet 0x7F "FLAC" + STREAMINFO): the packets are
//                   reassembled into a native FLAC stream for host_flac.hip; Vorbis
//                   (host_vorbis.hip); pages whose CRC fails are dropped.  Opus is a decoding
//                   error.
// MP3, AAC (MP4 / ADTS) and Opus are decoding errors that name the codec.  Parity
// with symphonia itself is unpinned (this image has no symphonia); tests/test_formats_decode.py
// writes each container from its specification and checks the reference's conversion bit for bit.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

bool sdsp_decode_flac(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_caf_alac(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_vorbis(const std::vector<std::vector<uint8_t>>& packets, int64_t last_granule, std::vector<float>* out,
                        uint32_t* sr, std::string* err);

namespace {

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
uint32_t le32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint64_t le64(const uint8_t* p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

// ITU-T G.711 expansions to 16-bit linear PCM (as host_decode.hip)
int16_t alaw16(uint8_t a) {
    a ^= 0x55;
    int t = (a & 0x0f) << 4;
    const int seg = (a & 0x70) >> 4;
    if (seg == 0)
        t += 8;
    else if (seg == 1)
        t += 0x108;
    else
        t = (t + 0x108) << (seg - 1);
    return (int16_t)((a & 0x80) ? t : -t);
}
int16_t ulaw16(uint8_t u) {
    u = ~u;
    int t = ((u & 0x0f) << 3) + 0x84;
    t <<= (u & 0x70) >> 4;
    return (int16_t)((u & 0x80) ? (0x84 - t) : (t - 0x84));
}

// One PCM sample layout; conv() gives the reference's f32 value of one channel sample.
struct Pcm {
    enum Kind { S16, S24, S32, F32, F64, ALAW, ULAW } kind = S16;
    bool big = true;
    int width = 2;
    float conv(const uint8_t* p) const {
        switch (kind) {
            case S16: return (float)(int16_t)(big ? be16(p) : (uint16_t)(p[0] | (p[1] << 8))) / 32768.0f;
            case S24: {
                int32_t v = big ? (int32_t)(((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2])
                                : (int32_t)(((uint32_t)p[2] << 16) | ((uint32_t)p[1] << 8) | p[0]);
                if (v & 0x800000) v -= 0x1000000;
                return (float)v / 8388608.0f;
            }
            case S32: return (float)(int32_t)(big ? be32(p) : le32(p)) / 2147483648.0f;
            case F32: {
                const uint32_t u = big ? be32(p) : le32(p);
                float f;
                std::memcpy(&f, &u, 4);
                return f;
            }
            case F64: {
                const uint64_t u = big ? be64(p) : le64(p);
                double d;
                std::memcpy(&d, &u, 8);
                return (float)d;
            }
            case ALAW: return (float)alaw16(p[0]) / 32768.0f;
            case ULAW: return (float)ulaw16(p[0]) / 32768.0f;
        }
        return 0.0f;
    }
};

// interleaved frames -> mono f32 (the examples' mix: sum from -0.0 in channel order, / channels)
void to_mono(const Pcm& pcm, int ch, const uint8_t* data, uint64_t frames, std::vector<float>* out) {
    out->resize(frames);
    const uint64_t stride = (uint64_t)pcm.width * (uint64_t)ch;
    for (uint64_t i = 0; i < frames; i++) {
        const uint8_t* p = data + i * stride;
        if (ch == 1) {
            (*out)[i] = pcm.conv(p);
        } else {
            float s = -0.0f;
            for (int c = 0; c < ch; c++) s = s + pcm.conv(p + (size_t)c * pcm.width);
            (*out)[i] = s / (float)ch;
        }
    }
}

bool fail(std::string* err, const std::string& m) {
    *err = m;
    return false;
}

// PCM sample layout of an integer width in bits (signed samples): 8 bits is symphonia's S8, which
// the examples' conversion does not handle
bool int_pcm(int bits, bool big, Pcm* pcm, std::string* err) {
    pcm->big = big;
    if (bits == 16) {
        pcm->kind = Pcm::S16, pcm->width = 2;
    } else if (bits == 24) {
        pcm->kind = Pcm::S24, pcm->width = 3;
    } else if (bits == 32) {
        pcm->kind = Pcm::S32, pcm->width = 4;
    } else if (bits == 8) {
        return fail(err, "Unsupported audio format");  // S8 buffers (examples/analyze_file.rs:171-174)
    } else {
        return fail(err, "unsupported PCM bits per sample " + std::to_string(bits));
    }
    return true;
}

// IEEE 754 80-bit extended (AIFF COMM sampleRate) -> integer rate
uint32_t ext80(const uint8_t* p) {
    const int e = ((p[0] & 0x7f) << 8) | p[1];
    const uint64_t m = be64(p + 2);
    if (m == 0 || (p[0] & 0x80)) return 0;
    const double v = std::ldexp((double)m, e - 16383 - 63);
    return v >= 1.0 && v < 4294967296.0 ? (uint32_t)v : 0;
}

}  // namespace

// AIFF / AIFF-C: FORM container, COMM (channels, frames, sample size, rate[, compression]), SSND
bool sdsp_decode_aiff(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err) {
    if (f.size() < 12) return fail(err, "malformed AIFF file");
    const bool aifc = std::memcmp(f.data() + 8, "AIFC", 4) == 0;
    int ch = 0, bits = 0;
    uint32_t rate = 0;
    char comp[4] = {'N', 'O', 'N', 'E'};
    bool have_comm = false;
    const uint8_t* data = nullptr;
    uint64_t data_len = 0;
    size_t pos = 12;
    while (pos + 8 <= f.size()) {
        const uint8_t* c = f.data() + pos;
        const uint64_t len = be32(c + 4);
        const uint64_t avail = f.size() - (pos + 8);
        if (std::memcmp(c, "COMM", 4) == 0) {
            if (len < 18 || len > avail || (aifc && len < 22)) return fail(err, "malformed COMM chunk");
            ch = (int16_t)be16(c + 8);
            bits = (int16_t)be16(c + 14);
            rate = ext80(c + 16);
            if (aifc) std::memcpy(comp, c + 26, 4);
            have_comm = true;
        } else if (std::memcmp(c, "SSND", 4) == 0) {
            if (len < 8) return fail(err, "malformed SSND chunk");
            const uint64_t off = be32(c + 8);
            const uint64_t body = (len <= avail ? len : avail);
            if (body < 8 + off) return fail(err, "malformed SSND chunk");
            data = c + 16 + off;
            data_len = body - 8 - off;
        }
        pos += 8 + len + (len & 1);
    }
    if (!have_comm) return fail(err, "missing COMM chunk");
    if (!data) return fail(err, "missing SSND chunk");
    if (ch <= 0) return fail(err, "zero channels");
    Pcm pcm;
    const std::string cs(comp, 4);
    if (cs == "NONE" || cs == "twos") {
        if (!int_pcm(bits, true, &pcm, err)) return false;
    } else if (cs == "sowt") {
        if (!int_pcm(bits, false, &pcm, err)) return false;
    } else if (cs == "fl32" || cs == "FL32") {
        pcm.kind = Pcm::F32, pcm.width = 4;
    } else if (cs == "fl64" || cs == "FL64") {
        pcm.kind = Pcm::F64, pcm.width = 8;
    } else if (cs == "alaw" || cs == "ALAW") {
        pcm.kind = Pcm::ALAW, pcm.width = 1;
    } else if (cs == "ulaw" || cs == "ULAW") {
        pcm.kind = Pcm::ULAW, pcm.width = 1;
    } else {
        return fail(err, "unsupported AIFF-C compression type '" + cs + "'");
    }
    to_mono(pcm, ch, data, data_len / ((uint64_t)pcm.width * (uint64_t)ch), out);
    *sr = rate ? rate : 44100u;
    return true;
}

// CAF: 'caff' header, 'desc' (rate f64, format id, flags, bytes / packet, frames / packet,
// channels, bits), 'data' (edit count + audio; size -1 = to the end of the file)
bool sdsp_decode_caf(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err) {
    if (f.size() < 8 || be16(f.data() + 4) != 1) return fail(err, "malformed CAF file");
    bool have_desc = false;
    double rate = 0.0;
    char fmt[4] = {0, 0, 0, 0};
    uint32_t flags = 0, bpp = 0, fpp = 0, ch = 0, bits = 0;
    const uint8_t* data = nullptr;
    uint64_t data_len = 0;
    size_t pos = 8;
    while (pos + 12 <= f.size()) {
        const uint8_t* c = f.data() + pos;
        const int64_t slen = (int64_t)be64(c + 4);
        const uint64_t avail = f.size() - (pos + 12);
        if (std::memcmp(c, "desc", 4) == 0) {
            if (slen < 32 || (uint64_t)slen > avail) return fail(err, "malformed desc chunk");
            const uint64_t rb = be64(c + 12);
            std::memcpy(&rate, &rb, 8);
            std::memcpy(fmt, c + 20, 4);
            flags = be32(c + 24);
            bpp = be32(c + 28);
            fpp = be32(c + 32);
            ch = be32(c + 36);
            bits = be32(c + 40);
            have_desc = true;
        } else if (std::memcmp(c, "data", 4) == 0) {
            const uint64_t body = (slen < 0 || (uint64_t)slen > avail) ? avail : (uint64_t)slen;
            if (body < 4) return fail(err, "malformed data chunk");
            data = c + 16;
            data_len = body - 4;
            if (slen < 0) break;  // the data chunk runs to the end of the file
        }
        if (slen < 0) break;
        pos += 12 + (uint64_t)slen;
    }
    if (!have_desc) return fail(err, "missing desc chunk");
    if (!data) return fail(err, "missing data chunk");
    if (ch == 0 || ch > 64) return fail(err, "unsupported channel count");
    const std::string fs(fmt, 4);
    Pcm pcm;
    if (fs == "lpcm") {
        const bool is_float = flags & 1u, little = flags & 2u;
        if (is_float) {
            if (bits == 32)
                pcm.kind = Pcm::F32, pcm.width = 4;
            else if (bits == 64)
                pcm.kind = Pcm::F64, pcm.width = 8;
            else
                return fail(err, "unsupported float bits per sample " + std::to_string(bits));
            pcm.big = !little;
        } else if (!int_pcm((int)bits, !little, &pcm, err)) {
            return false;
        }
        if (fpp != 1 || bpp != (uint32_t)pcm.width * ch) return fail(err, "unsupported CAF packet layout");
    } else if (fs == "alaw" || fs == "ulaw") {
        pcm.kind = fs == "alaw" ? Pcm::ALAW : Pcm::ULAW;
        pcm.width = 1;
    } else if (fs == "alac") {
        return sdsp_decode_caf_alac(f, out, sr, err);
    } else {
        return fail(err, "unsupported CAF format '" + fs + "'");
    }
    to_mono(pcm, (int)ch, data, data_len / ((uint64_t)pcm.width * ch), out);
    *sr = rate >= 1.0 && rate < 4294967296.0 ? (uint32_t)rate : 44100u;
    return true;
}

namespace {
// Ogg page CRC-32 (polynomial 0x04C11DB7, not reflected, initial 0, the CRC field read as 0)
uint32_t ogg_crc(const uint8_t* p, size_t n) {
    static uint32_t tab[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t r = i << 24;
            for (int k = 0; k < 8; k++) r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : r << 1;
            tab[i] = r;
        }
        init = true;
    }
    uint32_t crc = 0;
    for (size_t i = 0; i < n; i++) {
        const uint8_t b = (i >= 22 && i < 26) ? 0 : p[i];
        crc = (crc << 8) ^ tab[((crc >> 24) ^ b) & 0xFF];
    }
    return crc;
}
}  // namespace

// Ogg: the first logical stream's packets; the FLAC mapping is decoded, other codecs named
bool sdsp_decode_ogg(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err) {
    std::vector<std::vector<uint8_t>> packets;
    std::vector<uint8_t> cur;
    bool have_serial = false;
    uint32_t serial = 0;
    int64_t last_granule = -1;  // of the last page of the stream that completes a packet
    size_t pos = 0;
    while (pos + 27 <= f.size()) {
        const uint8_t* p = f.data() + pos;
        if (std::memcmp(p, "OggS", 4) != 0) {  // resynchronise on the next capture pattern
            pos++;
            continue;
        }
        const int nseg = p[26];
        if (pos + 27 + (size_t)nseg > f.size()) break;
        size_t body = 0;
        for (int i = 0; i < nseg; i++) body += p[27 + i];
        const size_t plen = 27 + (size_t)nseg + body;
        if (pos + plen > f.size()) break;
        if (ogg_crc(p, plen) != le32(p + 22)) {  // a damaged page: dropped with its partial packet
            cur.clear();
            pos++;
            continue;
        }
        const uint32_t s = le32(p + 14);
        if (!have_serial) {
            serial = s;
            have_serial = true;
        }
        if (s == serial) {
            const int64_t g = (int64_t)le64(p + 6);
            if (g != -1) last_granule = g;
            if (!(p[5] & 1)) cur.clear();  // not a continuation: no packet carries over
            const uint8_t* d = p + 27 + nseg;
            for (int i = 0; i < nseg; i++) {
                cur.insert(cur.end(), d, d + p[27 + i]);
                d += p[27 + i];
                if (p[27 + i] < 255) {
                    packets.push_back(std::move(cur));
                    cur.clear();
                }
            }
        }
        pos += plen;
    }
    if (packets.empty()) return fail(err, "no Ogg packets");
    const std::vector<uint8_t>& h = packets[0];
    if (h.size() >= 7 && h[0] == 0x01 && std::memcmp(h.data() + 1, "vorbis", 6) == 0)
        return sdsp_decode_vorbis(packets, last_granule, out, sr, err);
    if (h.size() >= 8 && std::memcmp(h.data(), "OpusHead", 8) == 0) return fail(err, "unsupported codec: Opus");
    if (!(h.size() >= 13 + 38 && h[0] == 0x7F && std::memcmp(h.data() + 1, "FLAC", 4) == 0 &&
          std::memcmp(h.data() + 9, "fLaC", 4) == 0))
        return fail(err, "unsupported Ogg stream");
    // native stream: "fLaC", STREAMINFO marked as the last metadata block, then the audio packets,
    // told from the header packets carrying the other metadata blocks by the frame sync code (the
    // first packet's header count may be 0, "unknown")
    std::vector<uint8_t> nat(h.begin() + 9, h.begin() + 13 + 38);
    nat[4] |= 0x80;
    for (size_t i = 1; i < packets.size(); i++) {
        const std::vector<uint8_t>& q = packets[i];
        if (q.size() >= 2 && q[0] == 0xFF && (q[1] & 0xFE) == 0xF8) nat.insert(nat.end(), q.begin(), q.end());
    }
    return sdsp_decode_flac(nat, out, sr, err);
}
