#include <cstdio>
#include <cstdint>
#include <cstdlib>
extern "C" int32_t sdsp_decode_audio_file(const char* path, float** samples, uint64_t* n_samples, uint32_t* sample_rate,
                                          char* err, uint64_t errlen);
extern "C" void sdsp_free_samples(float* samples);
int main(int argc, char** argv) {
    int ok = 0, bad = 0;
    for (int i = 1; i < argc; i++) {
        float* s = nullptr; uint64_t n = 0; uint32_t sr = 0; char err[256];
        if (sdsp_decode_audio_file(argv[i], &s, &n, &sr, err, sizeof err) == 0) { ok++; sdsp_free_samples(s); } else bad++;
    }
    std::printf("ok %d failed %d\n", ok, bad);
}
