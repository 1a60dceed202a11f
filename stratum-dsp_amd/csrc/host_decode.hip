// host_decode.hip — audio decode front-end exported through the C ABI (sdsp_decode_audio_file).
//
// The reference decodes with symphonia and converts every decoded buffer to mono f32 in its
// examples (examples/analyze_file.rs:25-180, examples/analyze_batch.rs:30-177):
//   F32 as is, F64 `as f32`, S16 `/ 32768.0`, S24 `i24 as f32 / 8388608.0`,
//   S32 `/ 2147483648.0`, U8 `(s - 128.0) / 128.0`;
//   more than one channel: the per-channel values summed in channel order (Iterator::sum, which
//   folds from -0.0) and divided by `channels as f32`.
// This front-end reads RIFF/WAVE (PCM, IEEE float, A-law, mu-law, IMA and Microsoft ADPCM, and
// WAVE_FORMAT_EXTENSIBLE with those sub-formats), which symphonia decodes into exactly those buffer
// types (A-law / mu-law / ADPCM to S16), FLAC (host_flac.hip; symphonia's S32 buffers), and AIFF /
// AIFF-C, CAF and Ogg FLAC (host_formats.hip), ALAC in CAF or MP4 (host_alac.hip), Ogg Vorbis
// (host_vorbis.hip) and Matroska / WebM with those codecs (host_mkv.hip).  A frame's
// mono value depends only on that frame, so packet boundaries do not matter.  Other codecs (MP3,
// AAC, Vorbis, Opus) are a decoding error that names the codec.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/stratum_hip.h"

bool sdsp_decode_flac(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_aiff(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_caf(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_ogg(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_mp4(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);
bool sdsp_decode_mkv(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);

namespace {

struct Fmt {
    uint16_t tag = 0, channels = 0, block_align = 0, bits = 0;
    uint32_t rate = 0;
    std::vector<int> ms_coef;  // Microsoft ADPCM coefficient pairs (fmt extension)
};

uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }

// ITU-T G.711 expansions to 16-bit linear PCM
int16_t alaw_to_s16(uint8_t a) {
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
int16_t ulaw_to_s16(uint8_t u) {
    u = ~u;
    int t = ((u & 0x0f) << 3) + 0x84;
    t <<= (u & 0x70) >> 4;
    return (int16_t)((u & 0x80) ? (0x84 - t) : (t - 0x84));
}

enum class Kind { U8, S16, S24, S32, F32, F64, ALAW, ULAW };

// one channel sample -> f32, the reference's per-type conversion
inline float conv(Kind k, const uint8_t* p) {
    switch (k) {
        case Kind::U8: return ((float)p[0] - 128.0f) / 128.0f;
        case Kind::S16: return (float)(int16_t)rd16(p) / 32768.0f;
        case Kind::S24: {
            int32_t v = (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16));
            if (v & 0x800000) v -= 0x1000000;
            return (float)v / 8388608.0f;
        }
        case Kind::S32: return (float)(int32_t)rd32(p) / 2147483648.0f;
        case Kind::F32: {
            float f;
            std::memcpy(&f, p, 4);
            return f;
        }
        case Kind::F64: {
            double d;
            std::memcpy(&d, p, 8);
            return (float)d;
        }
        case Kind::ALAW: return (float)alaw_to_s16(p[0]) / 32768.0f;
        case Kind::ULAW: return (float)ulaw_to_s16(p[0]) / 32768.0f;
    }
    return 0.0f;
}

bool fail(char* err, uint64_t errlen, const std::string& m) {
    if (err && errlen) std::snprintf(err, errlen, "%s", m.c_str());
    return false;
}

// ---- ADPCM in WAV (symphonia-codec-adpcm decodes both to S16 buffers) ----
// IMA ADPCM (WAVE tag 0x11, 4 bits): per block and channel a 4-byte header (predictor i16, step
// index u8, reserved), which is the block's first sample; then 4-byte words per channel in turn,
// 8 samples each, low nibble first.  A nibble n updates the predictor by +-((2 (n & 7) + 1) step)
// >> 3, clamped to i16, and the step index by the index table, clamped to [0, 88].
const int16_t IMA_STEP[89] = {7,     8,     9,     10,    11,    12,    13,    14,    16,    17,    19,    21,    23,
                              25,    28,    31,    34,    37,    41,    45,    50,    55,    60,    66,    73,    80,
                              88,    97,    107,   118,   130,   143,   157,   173,   190,   209,   230,   253,   279,
                              307,   337,   371,   408,   449,   494,   544,   598,   658,   724,   796,   876,   963,
                              1060,  1166,  1282,  1411,  1552,  1707,  1878,  2066,  2272,  2499,  2749,  3024,  3327,
                              3660,  4026,  4428,  4871,  5358,  5894,  6484,  7132,  7845,  8630,  9493,  10442, 11487,
                              12635, 13899, 15289, 16818, 18500, 20350, 22385, 24623, 27086, 29794, 32767};
const int IMA_INDEX[16] = {-1, -1, -1, -1, 2, 4, 6, 8, -1, -1, -1, -1, 2, 4, 6, 8};

struct ImaState {
    int pred = 0, idx = 0;
    int16_t nibble(int n) {
        const int step = IMA_STEP[idx];
        const int diff = ((2 * (n & 7) + 1) * step) >> 3;
        pred = (n & 8) ? pred - diff : pred + diff;
        pred = pred < -32768 ? -32768 : pred > 32767 ? 32767 : pred;
        idx += IMA_INDEX[n];
        idx = idx < 0 ? 0 : idx > 88 ? 88 : idx;
        return (int16_t)pred;
    }
};

// blocks of `ba` bytes -> interleaved S16 frames (a final partial block keeps its whole words)
bool ima_decode(const uint8_t* d, uint64_t n, int ch, int ba, std::vector<int16_t>* pcm, char* err, uint64_t errlen) {
    if (ch > 64) return fail(err, errlen, "unsupported channel count");
    if (ba < 4 * ch || (ba - 4 * ch) % (4 * ch) != 0) return fail(err, errlen, "malformed IMA ADPCM block alignment");
    std::vector<ImaState> st((size_t)ch);
    for (uint64_t b = 0; b + 4 * (uint64_t)ch <= n; b += (uint64_t)ba) {
        const uint8_t* p = d + b;
        const uint64_t len = n - b < (uint64_t)ba ? n - b : (uint64_t)ba;
        for (int c = 0; c < ch; c++) {
            st[c].pred = (int16_t)rd16(p + 4 * c);
            st[c].idx = p[4 * c + 2] > 88 ? 88 : p[4 * c + 2];
            pcm->push_back((int16_t)st[c].pred);
        }
        const uint64_t words = (len - 4 * (uint64_t)ch) / (4 * (uint64_t)ch);
        const uint8_t* q = p + 4 * ch;
        for (uint64_t w = 0; w < words; w++) {
            int16_t blk[8 * 64];
            for (int c = 0; c < ch; c++) {
                for (int j = 0; j < 4; j++) {
                    const uint8_t byte = q[(w * ch + c) * 4 + j];
                    blk[(2 * j) * ch + c] = st[c].nibble(byte & 15);
                    blk[(2 * j + 1) * ch + c] = st[c].nibble(byte >> 4);
                }
            }
            pcm->insert(pcm->end(), blk, blk + 8 * ch);
        }
    }
    return true;
}

// Microsoft ADPCM (WAVE tag 0x2): per block a header of predictor indices (u8 per channel), then
// deltas, sample1 and sample2 (i16 per channel each); sample2 and sample1 are the first two
// frames.  Then one nibble per channel sample, interleaved by channel, high nibble first:
// pred = (s1 c1 + s2 c2) / 256 (toward zero) + nibble (signed) * delta, clamped to i16;
// delta = max(16, (ADAPT[nibble] * delta) >> 8).  Coefficient pairs from the fmt extension.
const int MS_ADAPT[16] = {230, 230, 230, 230, 307, 409, 512, 614, 768, 614, 512, 409, 307, 230, 230, 230};

bool msadpcm_decode(const uint8_t* d, uint64_t n, int ch, int ba, const std::vector<int>& coef,
                    std::vector<int16_t>* pcm, char* err, uint64_t errlen) {
    if (ba < 7 * ch) return fail(err, errlen, "malformed MS ADPCM block alignment");
    const int ncoef = (int)coef.size() / 2;
    std::vector<int> c1((size_t)ch), c2((size_t)ch), delta((size_t)ch), s1((size_t)ch), s2((size_t)ch);
    for (uint64_t b = 0; b + 7 * (uint64_t)ch <= n; b += (uint64_t)ba) {
        const uint8_t* p = d + b;
        const uint64_t len = n - b < (uint64_t)ba ? n - b : (uint64_t)ba;
        for (int c = 0; c < ch; c++) {
            const int pi = p[c];
            if (pi >= ncoef) return fail(err, errlen, "MS ADPCM predictor index out of range");
            c1[c] = coef[2 * pi];
            c2[c] = coef[2 * pi + 1];
            delta[c] = (int16_t)rd16(p + ch + 2 * c);
            s1[c] = (int16_t)rd16(p + 3 * ch + 2 * c);
            s2[c] = (int16_t)rd16(p + 5 * ch + 2 * c);
        }
        for (int c = 0; c < ch; c++) pcm->push_back((int16_t)s2[c]);
        for (int c = 0; c < ch; c++) pcm->push_back((int16_t)s1[c]);
        int c = 0;
        for (uint64_t k = 7 * (uint64_t)ch; k < len; k++) {
            for (int half = 0; half < 2; half++) {
                const int nib = half == 0 ? p[k] >> 4 : p[k] & 15;
                const int sn = nib >= 8 ? nib - 16 : nib;
                // 64-bit predictor and adaptation: on corrupt nibbles delta grows without bound, and
                // (s1 c1 + s2 c2) reaches 2^31 at the extremes; delta is capped as FFmpeg's decoder
                // caps it (INT_MAX / 768), so every product stays well inside 64 bits
                int64_t pred = ((int64_t)s1[c] * c1[c] + (int64_t)s2[c] * c2[c]) / 256 + (int64_t)sn * delta[c];
                pred = pred < -32768 ? -32768 : pred > 32767 ? 32767 : pred;
                s2[c] = s1[c];
                s1[c] = (int)pred;
                int64_t nd = ((int64_t)MS_ADAPT[nib] * delta[c]) >> 8;
                nd = nd < 16 ? 16 : nd > INT32_MAX / 768 ? INT32_MAX / 768 : nd;
                delta[c] = (int)nd;
                pcm->push_back((int16_t)pred);
                c = c + 1 == ch ? 0 : c + 1;
            }
        }
        if (c != 0) pcm->resize(pcm->size() - (size_t)c);  // an incomplete frame (odd channel counts)
    }
    return true;
}

bool decode_wav(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, char* err, uint64_t errlen) {
    if (f.size() < 12 || std::memcmp(f.data(), "RIFF", 4) != 0 || std::memcmp(f.data() + 8, "WAVE", 4) != 0)
        return fail(err, errlen, "unsupported format: not a RIFF/WAVE file");
    Fmt fmt;
    bool have_fmt = false;
    const uint8_t* data = nullptr;
    uint64_t data_len = 0;
    size_t pos = 12;
    while (pos + 8 <= f.size()) {
        const uint8_t* c = f.data() + pos;
        const uint64_t len = rd32(c + 4);
        const uint64_t avail = f.size() - (pos + 8);
        if (std::memcmp(c, "fmt ", 4) == 0) {
            if (len < 16 || len > avail) return fail(err, errlen, "malformed fmt chunk");
            fmt.tag = rd16(c + 8);
            fmt.channels = rd16(c + 10);
            fmt.rate = rd32(c + 12);
            fmt.block_align = rd16(c + 20);
            fmt.bits = rd16(c + 22);
            if (fmt.tag == 0xFFFE) {  // WAVE_FORMAT_EXTENSIBLE: sub-format GUID's first two bytes
                if (len < 40) return fail(err, errlen, "malformed extensible fmt chunk");
                fmt.tag = rd16(c + 8 + 24);
            } else if (fmt.tag == 2) {  // cbSize, samples per block, coefficient count, pairs
                if (len < 22) return fail(err, errlen, "malformed MS ADPCM fmt chunk");
                const int nc = rd16(c + 8 + 20);
                if (nc < 1 || len < 22 + 4 * (uint64_t)nc) return fail(err, errlen, "malformed MS ADPCM fmt chunk");
                for (int i = 0; i < 2 * nc; i++) fmt.ms_coef.push_back((int16_t)rd16(c + 8 + 22 + 2 * i));
            }
            have_fmt = true;
        } else if (std::memcmp(c, "data", 4) == 0) {
            data = c + 8;
            data_len = len <= avail ? len : avail;  // a truncated file keeps its whole frames
            break;
        }
        pos += 8 + len + (len & 1);
    }
    if (!have_fmt) return fail(err, errlen, "missing fmt chunk");
    if (!data) return fail(err, errlen, "missing data chunk");
    if (fmt.channels == 0) return fail(err, errlen, "zero channels");
    Kind k;
    int width;
    if (fmt.tag == 1) {
        if (fmt.bits == 8)
            k = Kind::U8, width = 1;
        else if (fmt.bits == 16)
            k = Kind::S16, width = 2;
        else if (fmt.bits == 24)
            k = Kind::S24, width = 3;
        else if (fmt.bits == 32)
            k = Kind::S32, width = 4;
        else
            return fail(err, errlen, "unsupported PCM bits per sample " + std::to_string(fmt.bits));
    } else if (fmt.tag == 3) {
        if (fmt.bits == 32)
            k = Kind::F32, width = 4;
        else if (fmt.bits == 64)
            k = Kind::F64, width = 8;
        else
            return fail(err, errlen, "unsupported float bits per sample " + std::to_string(fmt.bits));
    } else if (fmt.tag == 6 && fmt.bits == 8) {
        k = Kind::ALAW, width = 1;
    } else if (fmt.tag == 7 && fmt.bits == 8) {
        k = Kind::ULAW, width = 1;
    } else if ((fmt.tag == 0x11 && fmt.bits == 4) || fmt.tag == 2) {
        std::vector<int16_t> pcm;
        const bool ok = fmt.tag == 0x11 ? ima_decode(data, data_len, fmt.channels, fmt.block_align, &pcm, err, errlen)
                                        : msadpcm_decode(data, data_len, fmt.channels, fmt.block_align, fmt.ms_coef,
                                                         &pcm, err, errlen);
        if (!ok) return false;
        const int ch = fmt.channels;
        const uint64_t frames = pcm.size() / (uint64_t)ch;
        out->resize(frames);
        for (uint64_t i = 0; i < frames; i++) {
            if (ch == 1) {
                (*out)[i] = (float)pcm[i] / 32768.0f;
            } else {
                float s = -0.0f;
                for (int c2 = 0; c2 < ch; c2++) s = s + (float)pcm[i * ch + c2] / 32768.0f;
                (*out)[i] = s / (float)ch;
            }
        }
        *sr = fmt.rate ? fmt.rate : 44100u;
        return true;
    } else {
        return fail(err, errlen, "unsupported WAVE format tag " + std::to_string(fmt.tag));
    }
    const uint64_t stride = (uint64_t)width * fmt.channels;
    if (fmt.block_align != 0 && fmt.block_align != stride) return fail(err, errlen, "unsupported block alignment");
    const uint64_t frames = data_len / stride;
    out->resize(frames);
    const int ch = fmt.channels;
    for (uint64_t i = 0; i < frames; i++) {
        const uint8_t* p = data + i * stride;
        if (ch == 1) {
            (*out)[i] = conv(k, p);
        } else {
            float s = -0.0f;
            for (int c2 = 0; c2 < ch; c2++) s = s + conv(k, p + c2 * width);
            (*out)[i] = s / (float)ch;
        }
    }
    *sr = fmt.rate ? fmt.rate : 44100u;  // codec_params.sample_rate.unwrap_or(44100)
    return true;
}

}  // namespace

namespace {
int32_t decode_audio_file(const char* path, float** samples, uint64_t* n_samples, uint32_t* sample_rate, char* err,
                          uint64_t errlen) {
    if (err && errlen) err[0] = 0;
    if (!path || !samples || !n_samples || !sample_rate) return SDSP_ERR_INVALID_INPUT;
    *samples = nullptr;
    *n_samples = 0;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) {
        fail(err, errlen, std::string("cannot open ") + path);
        return SDSP_ERR_DECODING;
    }
    std::vector<uint8_t> buf;
    uint8_t chunk[1 << 16];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof chunk, fp)) > 0) buf.insert(buf.end(), chunk, chunk + got);
    std::fclose(fp);
    std::vector<float> mono;
    uint32_t sr = 0;
    auto magic = [&](size_t off, const char* m) {
        const size_t n = std::strlen(m);
        return buf.size() >= off + n && std::memcmp(buf.data() + off, m, n) == 0;
    };
    // an ID3v2 tag (10-byte header, syncsafe size) may precede FLAC or MP3 data
    size_t id3 = 0;
    if (magic(0, "ID3") && buf.size() >= 10)
        id3 = 10 + (((size_t)(buf[6] & 0x7f) << 21) | ((size_t)(buf[7] & 0x7f) << 14) | ((size_t)(buf[8] & 0x7f) << 7) |
                    (size_t)(buf[9] & 0x7f));
    std::string why;
    bool ok;
    if (magic(0, "fLaC") || (id3 && magic(id3, "fLaC"))) {
        ok = sdsp_decode_flac(buf, &mono, &sr, &why);
    } else if (magic(0, "FORM") && (magic(8, "AIFF") || magic(8, "AIFC"))) {
        ok = sdsp_decode_aiff(buf, &mono, &sr, &why);
    } else if (magic(0, "caff")) {
        ok = sdsp_decode_caf(buf, &mono, &sr, &why);
    } else if (magic(0, "OggS")) {
        ok = sdsp_decode_ogg(buf, &mono, &sr, &why);
    } else if (buf.size() >= 4 && buf[0] == 0x1A && buf[1] == 0x45 && buf[2] == 0xDF && buf[3] == 0xA3) {
        ok = sdsp_decode_mkv(buf, &mono, &sr, &why);
    } else if (magic(4, "ftyp")) {
        ok = sdsp_decode_mp4(buf, &mono, &sr, &why);
    } else if (id3 || (buf.size() >= 2 && buf[0] == 0xFF && (buf[1] & 0xE0) == 0xE0)) {
        ok = false, why = (buf.size() >= 2 && !id3 && (buf[1] & 0xF6) == 0xF0) ? "unsupported codec: AAC (ADTS)"
                                                                             : "unsupported codec: MPEG audio (MP1/MP2/MP3)";
    } else {
        if (!decode_wav(buf, &mono, &sr, err, errlen)) return SDSP_ERR_DECODING;
        ok = true;
    }
    if (!ok) {
        fail(err, errlen, why);
        return SDSP_ERR_DECODING;
    }
    float* p = (float*)std::malloc(std::max<size_t>(mono.size(), 1) * sizeof(float));
    if (!p) return SDSP_ERR_PROCESSING;
    if (!mono.empty()) std::memcpy(p, mono.data(), mono.size() * sizeof(float));
    *samples = p;
    *n_samples = mono.size();
    *sample_rate = sr;
    return SDSP_OK;
}
}  // namespace

// No exception leaves the C ABI: sizes a damaged header declares can make an allocation fail
// (std::bad_alloc / std::length_error) inside any of the decoders.
extern "C" int32_t sdsp_decode_audio_file(const char* path, float** samples, uint64_t* n_samples, uint32_t* sample_rate,
                                          char* err, uint64_t errlen) {
    try {
        return decode_audio_file(path, samples, n_samples, sample_rate, err, errlen);
    } catch (const std::exception& e) {
        fail(err, errlen, std::string("decoding failed: ") + e.what());
    } catch (...) {
        fail(err, errlen, "decoding failed");
    }
    if (samples) *samples = nullptr;
    if (n_samples) *n_samples = 0;
    return SDSP_ERR_DECODING;
}

extern "C" void sdsp_free_samples(float* samples) { std::free(samples); }
