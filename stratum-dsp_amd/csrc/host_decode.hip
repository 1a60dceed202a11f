// host_decode.hip — audio decode front-end exported through the C ABI (sdsp_decode_audio_file).
//
// The reference decodes with symphonia and converts every decoded buffer to mono f32 in its
// examples (examples/analyze_file.rs:25-180, examples/analyze_batch.rs:30-177):
//   F32 as is, F64 `as f32`, S16 `/ 32768.0`, S24 `i24 as f32 / 8388608.0`,
//   S32 `/ 2147483648.0`, U8 `(s - 128.0) / 128.0`;
//   more than one channel: the per-channel values summed in channel order (Iterator::sum, which
//   folds from -0.0) and divided by `channels as f32`.
// This front-end reads RIFF/WAVE (PCM, IEEE float, A-law, mu-law, and WAVE_FORMAT_EXTENSIBLE
// with those sub-formats), which symphonia decodes into exactly those buffer types (A-law /
// mu-law expand to S16, ITU-T G.711), and FLAC (host_flac.hip; symphonia's S32 buffers).  A
// frame's mono value depends only on that frame, so packet boundaries do not matter.  Other
// containers and codecs (MP3, AAC, Ogg Vorbis, ALAC, ...) are a decoding error.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/stratum_hip.h"

bool sdsp_decode_flac(const std::vector<uint8_t>& f, std::vector<float>* out, uint32_t* sr, std::string* err);

namespace {

struct Fmt {
    uint16_t tag = 0, channels = 0, block_align = 0, bits = 0;
    uint32_t rate = 0;
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

extern "C" int32_t sdsp_decode_audio_file(const char* path, float** samples, uint64_t* n_samples, uint32_t* sample_rate,
                                          char* err, uint64_t errlen) {
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
    const bool flac = (buf.size() >= 4 && std::memcmp(buf.data(), "fLaC", 4) == 0) ||
                      (buf.size() >= 3 && std::memcmp(buf.data(), "ID3", 3) == 0);
    if (flac) {
        std::string why;
        if (!sdsp_decode_flac(buf, &mono, &sr, &why)) {
            fail(err, errlen, why);
            return SDSP_ERR_DECODING;
        }
    } else if (!decode_wav(buf, &mono, &sr, err, errlen)) {
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

extern "C" void sdsp_free_samples(float* samples) { std::free(samples); }
