// pipeline.hip — analyze_audio on the GPU (placeholder entry points; filled in by the pipeline).
#include <cstdio>
#include <cstring>

#include "sdsp_runtime.hpp"

extern "C" {
int32_t sdsp_analyze_audio(const float*, uint64_t, uint32_t, const sdsp_config*, sdsp_result* out, char* err,
                           uint64_t errlen) {
    if (out) std::memset(out, 0, sizeof(*out));
    if (err && errlen) std::snprintf(err, errlen, "Not implemented: pipeline");
    return SDSP_ERR_NOT_IMPLEMENTED;
}
int32_t sdsp_analyze_batch(const float* const*, const uint64_t*, uint64_t, uint32_t, const sdsp_config*, uint32_t,
                           sdsp_result*) {
    return SDSP_ERR_NOT_IMPLEMENTED;
}
int32_t sdsp_analyze_batch_device(const float*, const uint64_t*, const uint64_t*, uint64_t, uint32_t,
                                  const sdsp_config*, int32_t, void*, sdsp_result*) {
    return SDSP_ERR_NOT_IMPLEMENTED;
}
int32_t sdsp_generate_synthetic(float*, uint64_t, uint64_t, uint32_t, uint64_t, int32_t, int32_t, void*, float*,
                                int32_t*) {
    return SDSP_ERR_NOT_IMPLEMENTED;
}
}
