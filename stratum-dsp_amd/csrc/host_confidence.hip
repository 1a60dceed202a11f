// host_confidence.hip — host-side result post-processing exported through the C ABI:
//
//   sdsp_compute_confidence   compute_confidence            src/analysis/confidence.rs:121-297
//   sdsp_key_name             Key::name                     src/analysis/result.rs:31-39
//
// Pure f32 scalar code on the host, in the reference's operation order (-ffp-contract=off).
#include <cstdio>
#include <cstring>

#include "../../include/stratum_hip.h"

namespace {

// f32::clamp (NaN stays NaN)
float clampf(float x, float lo, float hi) {
    if (x < lo) return lo;
    if (x > hi) return hi;
    return x;
}

bool any_warning_contains(const sdsp_result* r, const char* const* needles, int n) {
    for (uint64_t i = 0; i < r->n_warnings; i++) {
        const char* w = r->warnings ? r->warnings[i] : nullptr;
        if (!w) continue;
        for (int k = 0; k < n; k++)
            if (std::strstr(w, needles[k])) return true;
    }
    return false;
}

// compute_bpm_confidence (confidence.rs:247-268)
float bpm_confidence(const sdsp_result* r) {
    if (r->bpm <= 0.0f) return 0.0f;
    const float base = clampf(r->bpm_confidence, 0.0f, 1.0f);
    static const char* const k[] = {"BPM"};
    return any_warning_contains(r, k, 1) ? base * 0.7f : base;
}

// compute_key_confidence (confidence.rs:276-307)
float key_confidence(const sdsp_result* r) {
    if (r->key_confidence <= 0.0f) return 0.0f;
    const float base = clampf(r->key_confidence, 0.0f, 1.0f);
    const float clarity_adj = r->key_clarity < 0.2f ? 0.6f : r->key_clarity < 0.5f ? 0.85f : 1.0f;
    static const char* const k[] = {"key", "Key", "tonality"};
    const float warning_adj = any_warning_contains(r, k, 3) ? 0.7f : 1.0f;
    return base * clarity_adj * warning_adj;
}

}  // namespace

extern "C" int32_t sdsp_compute_confidence(const sdsp_result* r, sdsp_confidence* out) {
    if (!r || !out) return SDSP_ERR_INVALID_INPUT;
    std::memset(out, 0, sizeof(*out));
    const float b = bpm_confidence(r);
    const float k = key_confidence(r);
    const float g = clampf(r->grid_stability, 0.0f, 1.0f);
    float overall;
    if (b > 0.0f && k > 0.0f)
        overall = clampf(b * 0.4f + k * 0.3f + g * 0.3f, 0.0f, 1.0f);
    else if (b > 0.0f)
        overall = b * 0.6f;
    else if (k > 0.0f)
        overall = k * 0.6f;
    else
        overall = 0.0f;
    out->bpm_confidence = b;
    out->key_confidence = k;
    out->grid_stability = g;
    out->overall_confidence = overall;
    // result.metadata.flags (analyze_audio pushes at most WeakTonality), then the new ones
    for (int i = 0; i < 4; i++)
        if (r->flags & (1u << i)) out->flag_list[out->n_flags++] = i;
    if (b < 0.3f) out->flag_list[out->n_flags++] = 0;  // MultimodalBpm
    if (k < 0.2f) out->flag_list[out->n_flags++] = 1;  // WeakTonality
    if (g < 0.3f) out->flag_list[out->n_flags++] = 2;  // TempoVariation
    return SDSP_OK;
}

extern "C" int32_t sdsp_key_name(int32_t key_mode, uint32_t key_tonic, char* buf, uint64_t buflen) {
    static const char* const names[12] = {"C", "C#", "D", "D#", "E", "F", "F#", "G", "G#", "A", "A#", "B"};
    char tmp[8];
    const int n = std::snprintf(tmp, sizeof tmp, "%s%s", names[key_tonic % 12], key_mode == 1 ? "m" : "");
    if (buf && buflen) std::snprintf(buf, buflen, "%s", tmp);
    return n;
}
