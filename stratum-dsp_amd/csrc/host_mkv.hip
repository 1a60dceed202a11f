// host_mkv.hip — Matroska / WebM audio for the decode front-end (symphonia's MKV reader,
// Cargo.toml:15 features = ["all"]): the EBML structure (Segment, Tracks / TrackEntry, Cluster,
// SimpleBlock and BlockGroup / Block with Xiph, EBML or fixed-size lacing; unknown-size Segment
// and Cluster elements), the first audio track's frames in file order, handed to the codec:
//   A_PCM/INT/LIT, A_PCM/INT/BIG (16 / 24 / 32 bits; 8 bits unsigned, as WAVE), A_PCM/FLOAT/IEEE
//   (32 / 64 bits), A_FLAC (CodecPrivate "fLaC" + metadata, then the frames: host_flac.hip),
//   A_VORBIS (CodecPrivate: the three Xiph-laced headers; host_vorbis.hip), A_ALAC
//   (CodecPrivate: the ALAC cookie; host_alac.hip).
// A_MPEG/L*, A_AAC and A_OPUS are decoding errors that name the codec.  Samples go through the
// examples' conversion (examples/analyze_file.rs:25-180); parity with symphonia is unpinned
// (tests/test_mkv_decode.py writes the files from the Matroska specification).
#include <cstring>
#include <string>
#include <vector>

bool sdsp_decode_flac(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_vorbis(const std::vector<std::vector<uint8_t>>& packets, int64_t last_granule, std::vector<float>* out,
                        uint32_t* sr, std::string* err);
bool sdsp_decode_alac_packets(const std::vector<uint8_t>& cookie, const std::vector<std::vector<uint8_t>>& packets,
                              std::vector<float>* out, uint32_t* sr, std::string* err);

namespace {

bool fail(std::string* err, const std::string& m) {
    *err = m;
    return false;
}

// EBML variable-length integers: an element ID keeps its length marker, a size drops it (all
// value bits set = unknown size)
bool read_id(const uint8_t* p, size_t n, size_t* pos, uint32_t* id) {
    if (*pos >= n) return false;
    const uint8_t b = p[*pos];
    int len = 1;
    while (len <= 4 && !(b & (0x80 >> (len - 1)))) len++;
    if (len > 4 || *pos + (size_t)len > n) return false;
    uint32_t v = 0;
    for (int i = 0; i < len; i++) v = (v << 8) | p[*pos + (size_t)i];
    *pos += (size_t)len;
    *id = v;
    return true;
}
constexpr uint64_t UNKNOWN = ~0ull;
bool read_size(const uint8_t* p, size_t n, size_t* pos, uint64_t* sz) {
    if (*pos >= n) return false;
    const uint8_t b = p[*pos];
    int len = 1;
    while (len <= 8 && !(b & (0x80 >> (len - 1)))) len++;
    if (len > 8 || *pos + (size_t)len > n) return false;
    uint64_t v = b & (0xFF >> len);
    bool all = v == (uint64_t)(0xFF >> len);
    for (int i = 1; i < len; i++) {
        v = (v << 8) | p[*pos + (size_t)i];
        all = all && p[*pos + (size_t)i] == 0xFF;
    }
    *pos += (size_t)len;
    *sz = all ? UNKNOWN : v;
    return true;
}
uint64_t uint_be(const uint8_t* p, uint64_t n) {
    uint64_t v = 0;
    for (uint64_t i = 0; i < n && i < 8; i++) v = (v << 8) | p[i];
    return v;
}
double float_be(const uint8_t* p, uint64_t n) {
    if (n == 4) {
        const uint32_t u = (uint32_t)uint_be(p, 4);
        float f;
        std::memcpy(&f, &u, 4);
        return f;
    }
    if (n == 8) {
        const uint64_t u = uint_be(p, 8);
        double d;
        std::memcpy(&d, &u, 8);
        return d;
    }
    return 0.0;
}

struct Track {
    uint64_t number = 0, type = 0, channels = 1, bits = 0;
    double rate = 8000.0;  // the Matroska default SamplingFrequency
    std::string codec;
    std::vector<uint8_t> priv;
};

constexpr uint32_t ID_SEGMENT = 0x18538067, ID_TRACKS = 0x1654AE6B, ID_TRACKENTRY = 0xAE, ID_TRACKNUMBER = 0xD7,
                   ID_TRACKTYPE = 0x83, ID_CODECID = 0x86, ID_CODECPRIVATE = 0x63A2, ID_AUDIO = 0xE1,
                   ID_SAMPLINGFREQ = 0xB5, ID_CHANNELS = 0x9F, ID_BITDEPTH = 0x6264, ID_CLUSTER = 0x1F43B675,
                   ID_SIMPLEBLOCK = 0xA3, ID_BLOCKGROUP = 0xA0, ID_BLOCK = 0xA1;

bool is_top_level(uint32_t id) {  // the Segment's children: an unknown-size Cluster ends at one
    return id == ID_CLUSTER || id == ID_TRACKS || id == 0x114D9B74 || id == 0x1549A966 || id == 0x1C53BB6B ||
           id == 0x1254C367 || id == 0x1941A469 || id == 0x1043A770;
}

// the frames of one Block / SimpleBlock body, lacing undone
bool block_frames(const uint8_t* p, uint64_t n, uint64_t want_track, std::vector<std::vector<uint8_t>>* frames) {
    size_t pos = 0;
    uint64_t track;
    if (!read_size(p, (size_t)n, &pos, &track) || pos + 3 > n) return false;
    if (track != want_track) return true;
    const uint8_t flags = p[pos + 2];
    pos += 3;
    const int lacing = (flags >> 1) & 3;
    if (lacing == 0) {
        frames->emplace_back(p + pos, p + n);
        return true;
    }
    if (pos >= n) return false;
    const int count = p[pos++] + 1;
    std::vector<uint64_t> sizes;
    if (lacing == 1) {  // Xiph: 255-sums for all but the last
        for (int i = 0; i < count - 1; i++) {
            uint64_t s = 0;
            while (true) {
                if (pos >= n) return false;
                const uint8_t b = p[pos++];
                s += b;
                if (b < 255) break;
            }
            sizes.push_back(s);
        }
    } else if (lacing == 3) {  // EBML: the first size, then signed differences
        uint64_t s;
        if (!read_size(p, (size_t)n, &pos, &s) || s == UNKNOWN) return false;
        sizes.push_back(s);
        for (int i = 1; i < count - 1; i++) {
            const size_t st = pos;
            uint64_t raw;
            if (!read_size(p, (size_t)n, &pos, &raw) || raw == UNKNOWN) return false;
            const int len = (int)(pos - st);
            const int64_t bias = ((int64_t)1 << (7 * len - 1)) - 1;
            const int64_t v = (int64_t)sizes.back() + ((int64_t)raw - bias);
            if (v < 0) return false;
            sizes.push_back((uint64_t)v);
        }
    } else {  // fixed: equal sizes
        const uint64_t rest = n - pos;
        if (rest % (uint64_t)count) return false;
        for (int i = 0; i < count - 1; i++) sizes.push_back(rest / (uint64_t)count);
    }
    // every laced size is checked against the bytes left, so the running sum cannot wrap
    uint64_t used = 0;
    for (uint64_t s : sizes) {
        if (s > n - pos - used) return false;
        used += s;
    }
    sizes.push_back(n - pos - used);
    for (uint64_t s : sizes) {
        frames->emplace_back(p + pos, p + pos + s);
        pos += s;
    }
    return true;
}

void parse_track(const uint8_t* p, uint64_t n, Track* t) {
    size_t pos = 0;
    while (pos < n) {
        uint32_t id;
        uint64_t sz;
        if (!read_id(p, (size_t)n, &pos, &id) || !read_size(p, (size_t)n, &pos, &sz) || sz == UNKNOWN || sz > n - pos) return;
        const uint8_t* b = p + pos;
        if (id == ID_TRACKNUMBER) t->number = uint_be(b, sz);
        else if (id == ID_TRACKTYPE) t->type = uint_be(b, sz);
        else if (id == ID_CODECID) t->codec.assign((const char*)b, (size_t)sz), t->codec = t->codec.c_str();
        else if (id == ID_CODECPRIVATE) t->priv.assign(b, b + sz);
        else if (id == ID_AUDIO) {
            size_t q = 0;
            while (q < sz) {
                uint32_t id2;
                uint64_t s2;
                if (!read_id(b, (size_t)sz, &q, &id2) || !read_size(b, (size_t)sz, &q, &s2) || s2 == UNKNOWN || s2 > sz - q) break;
                if (id2 == ID_SAMPLINGFREQ) t->rate = float_be(b + q, s2);
                else if (id2 == ID_CHANNELS) t->channels = uint_be(b + q, s2);
                else if (id2 == ID_BITDEPTH) t->bits = uint_be(b + q, s2);
                q += s2;
            }
        }
        pos += sz;
    }
}

}  // namespace

bool sdsp_decode_mkv(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err) {
    const uint8_t* p = f.data();
    const size_t n = f.size();
    size_t pos = 0;
    uint32_t id;
    uint64_t sz;
    // EBML header, then the Segment
    if (!read_id(p, n, &pos, &id) || id != 0x1A45DFA3 || !read_size(p, n, &pos, &sz) || sz == UNKNOWN || sz > n - pos)
        return fail(err, "malformed Matroska file");
    pos += sz;
    if (!read_id(p, n, &pos, &id) || id != ID_SEGMENT || !read_size(p, n, &pos, &sz)) return fail(err, "missing Matroska segment");
    const size_t seg_end = sz == UNKNOWN || sz > n - pos ? n : pos + (size_t)sz;
    std::vector<Track> tracks;
    int audio_idx = -1;  // the first audio track
    std::vector<std::vector<uint8_t>> frames;
    // walk the Segment's children; Cluster children are walked in place (sizes may be unknown)
    std::vector<size_t> ends{seg_end};
    while (pos < seg_end) {
        while (ends.size() > 1 && pos >= ends.back()) ends.pop_back();
        if (!read_id(p, n, &pos, &id) || !read_size(p, n, &pos, &sz)) break;
        if (ends.size() > 1 && is_top_level(id)) ends.pop_back();  // an unknown-size Cluster ends here
        const size_t lim = ends.back();
        if (id == ID_CLUSTER) {
            ends.push_back(sz == UNKNOWN || sz > lim - pos ? lim : pos + (size_t)sz);
            continue;  // descend
        }
        if (sz == UNKNOWN || sz > lim - pos) return fail(err, "malformed Matroska element");
        if (id == ID_TRACKS) {
            size_t q = pos;
            while (q < pos + sz) {
                uint32_t id2;
                uint64_t s2;
                if (!read_id(p, pos + (size_t)sz, &q, &id2) || !read_size(p, pos + (size_t)sz, &q, &s2) || s2 == UNKNOWN ||
                    s2 > pos + sz - q)
                    break;
                if (id2 == ID_TRACKENTRY) {
                    Track t;
                    parse_track(p + q, s2, &t);
                    tracks.push_back(t);
                }
                q += s2;
            }
            for (size_t k = 0; k < tracks.size() && audio_idx < 0; k++)
                if (tracks[k].type == 2) audio_idx = (int)k;
        } else if (audio_idx >= 0 && (id == ID_SIMPLEBLOCK || id == ID_BLOCKGROUP)) {
            const uint64_t tn = tracks[(size_t)audio_idx].number;
            if (id == ID_SIMPLEBLOCK) {
                if (!block_frames(p + pos, sz, tn, &frames)) return fail(err, "malformed Matroska block");
            } else {
                size_t q = pos;
                while (q < pos + sz) {
                    uint32_t id2;
                    uint64_t s2;
                    if (!read_id(p, pos + (size_t)sz, &q, &id2) || !read_size(p, pos + (size_t)sz, &q, &s2) || s2 == UNKNOWN ||
                        s2 > pos + sz - q)
                        break;
                    if (id2 == ID_BLOCK && !block_frames(p + q, s2, tn, &frames))
                        return fail(err, "malformed Matroska block");
                    q += s2;
                }
            }
        }
        pos += sz;
    }
    if (audio_idx < 0) return fail(err, "no Matroska audio track");
    const Track& t = tracks[(size_t)audio_idx];
    const std::string& c = t.codec;
    const int ch = (int)t.channels;
    if (c == "A_FLAC") {
        std::vector<uint8_t> nat(t.priv);
        for (const auto& fr : frames) nat.insert(nat.end(), fr.begin(), fr.end());
        return sdsp_decode_flac(nat, out, sr, err);
    }
    if (c == "A_VORBIS") {  // CodecPrivate: 0x02, two Xiph-laced sizes, then the three headers
        const std::vector<uint8_t>& v = t.priv;
        if (v.size() < 3 || v[0] != 2) return fail(err, "malformed Vorbis CodecPrivate");
        size_t q = 1;
        uint64_t s[2] = {0, 0};
        for (int i = 0; i < 2; i++) {
            while (true) {
                if (q >= v.size()) return fail(err, "malformed Vorbis CodecPrivate");
                const uint8_t b = v[q++];
                s[i] += b;
                if (b < 255) break;
            }
        }
        if (s[0] + s[1] > v.size() - q) return fail(err, "malformed Vorbis CodecPrivate");
        std::vector<std::vector<uint8_t>> pk;
        pk.emplace_back(v.begin() + (long)q, v.begin() + (long)(q + s[0]));
        pk.emplace_back(v.begin() + (long)(q + s[0]), v.begin() + (long)(q + s[0] + s[1]));
        pk.emplace_back(v.begin() + (long)(q + s[0] + s[1]), v.end());
        pk.insert(pk.end(), frames.begin(), frames.end());
        return sdsp_decode_vorbis(pk, -1, out, sr, err);
    }
    if (c == "A_ALAC") return sdsp_decode_alac_packets(t.priv, frames, out, sr, err);
    if (c.rfind("A_PCM/", 0) == 0) {
        const bool fl = c == "A_PCM/FLOAT/IEEE", big = c == "A_PCM/INT/BIG";
        if (!fl && !big && c != "A_PCM/INT/LIT") return fail(err, "unsupported codec: " + c);
        const int bits = (int)t.bits, w = bits / 8;
        if (ch < 1 || bits % 8 || (fl && bits != 32 && bits != 64) || (!fl && (bits < 8 || bits > 32)))
            return fail(err, "unsupported PCM layout in Matroska");
        std::vector<uint8_t> data;
        for (const auto& fr : frames) data.insert(data.end(), fr.begin(), fr.end());
        const size_t frames_n = data.size() / ((size_t)w * (size_t)ch);
        out->resize(frames_n);
        auto conv = [&](const uint8_t* q) -> float {
            uint64_t u = 0;
            for (int i = 0; i < w; i++) u |= (uint64_t)q[big ? w - 1 - i : i] << (8 * i);
            if (fl) {
                if (w == 4) {
                    const uint32_t u32 = (uint32_t)u;
                    float f2;
                    std::memcpy(&f2, &u32, 4);
                    return f2;
                }
                double d;
                std::memcpy(&d, &u, 8);
                return (float)d;
            }
            if (bits == 8) return ((float)(uint8_t)u - 128.0f) / 128.0f;
            int64_t s = (int64_t)u;
            if (u >> (bits - 1)) s -= (int64_t)1 << bits;
            if (bits == 16) return (float)s / 32768.0f;
            if (bits == 24) return (float)s / 8388608.0f;
            return (float)(int32_t)s / 2147483648.0f;
        };
        for (size_t i = 0; i < frames_n; i++) {
            const uint8_t* q = data.data() + i * (size_t)w * (size_t)ch;
            if (ch == 1) {
                (*out)[i] = conv(q);
            } else {
                float s = -0.0f;
                for (int k = 0; k < ch; k++) s = s + conv(q + (size_t)k * (size_t)w);
                (*out)[i] = s / (float)ch;
            }
        }
        *sr = t.rate >= 1.0 && t.rate < 4294967296.0 ? (uint32_t)t.rate : 44100u;
        return true;
    }
    if (c.rfind("A_MPEG/", 0) == 0) return fail(err, "unsupported codec: MPEG audio (" + c + ")");
    if (c.rfind("A_AAC", 0) == 0) return fail(err, "unsupported codec: AAC (" + c + ")");
    return fail(err, "unsupported codec: " + c);
}
