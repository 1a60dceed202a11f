// analyze_file — single-file front-end with the reference example's interface and output
// (examples/analyze_file.rs): decode, AnalysisConfig::default() plus the command-line flags,
// analyze_audio on the GPU through the C ABI, compute_confidence, then the same JSON or
// human-readable report.
//
//   analyze_file <audio_file> [--json] [--debug] [flags of examples/analyze_file.rs]
#include <chrono>

#include "cli_common.hpp"

using namespace sdsp_cli;

int main(int argc, char** argv) {
    Args args(argv, argv + argc);
    if (args.size() < 2) {
        std::fprintf(stderr,
                     "Usage: %s <audio_file> [--json] [--debug] [--debug-track-id ID] [--debug-gt-bpm X] "
                     "[--no-preprocess] [--no-normalize] [--no-trim] [--no-onset-consensus] [--force-legacy-bpm] "
                     "[--bpm-fusion] [--no-tempogram-multi-res] [...]  (flags as examples/analyze_file.rs)\n",
                     args[0].c_str());
        return 1;
    }
    const std::string& path = args[1];
    const bool json = has(args, "--json");
    const bool debug = has(args, "--debug");

    float* samples = nullptr;
    uint64_t n = 0;
    uint32_t sr = 0;
    char err[512];
    if (sdsp_decode_audio_file(path.c_str(), &samples, &n, &sr, err, sizeof err) != 0) {
        std::fprintf(stderr, "Error: %s\n", err);
        return 1;
    }
    if (n == 0) {
        std::fprintf(stderr, "ERROR: No audio samples decoded from file\n");
        sdsp_free_samples(samples);
        return 1;
    }
    sdsp_config cfg;
    sdsp_config_default(&cfg);
    ConfigStore store;
    apply_flags(args, &cfg, &store);

    if (debug) {
        std::printf("=== DEBUG MODE ===\n");
        std::printf("Audio file: %s\n", path.c_str());
        std::printf("Samples: %llu, Sample rate: %u Hz\n", (unsigned long long)n, sr);
        std::printf("Duration: %.2f seconds\n", (double)((float)n / (float)sr));
        std::printf("\n");
    }

    sdsp_result res;
    const int32_t st = sdsp_analyze_audio(samples, n, sr, &cfg, &res, err, sizeof err);
    sdsp_free_samples(samples);
    if (st != 0) {
        std::fprintf(stderr, "ERROR: Analysis failed: %s\n", err);
        return 1;
    }
    sdsp_confidence conf;
    sdsp_compute_confidence(&res, &conf);
    const std::string key = key_name(res);
    if (json) {
        std::printf("{\n");
        std::printf("  \"bpm\": %.2f,\n", (double)res.bpm);
        std::printf("  \"bpm_confidence\": %.2f,\n", (double)conf.bpm_confidence);
        std::printf("  \"key\": \"%s\",\n", key.c_str());
        std::printf("  \"key_confidence\": %.2f,\n", (double)conf.key_confidence);
        std::printf("  \"key_clarity\": %.2f,\n", (double)res.key_clarity);
        std::printf("  \"grid_stability\": %.2f,\n", (double)res.grid_stability);
        const int8_t tr[4] = {res.tempogram_multi_res_triggered, res.tempogram_multi_res_used,
                              res.tempogram_percussive_triggered, res.tempogram_percussive_used};
        const char* tn[4] = {"tempogram_multi_res_triggered", "tempogram_multi_res_used",
                             "tempogram_percussive_triggered", "tempogram_percussive_used"};
        for (int i = 0; i < 4; i++)
            if (tr[i] >= 0) std::printf("  \"%s\": %s,\n", tn[i], tr[i] ? "true" : "false");
        if (res.has_tempogram_candidates) {
            std::printf("  \"bpm_candidates\": [\n");
            for (uint64_t i = 0; i < res.n_tempogram_candidates; i++) {
                const sdsp_tempo_candidate& c = res.tempogram_candidates[i];
                std::printf("    { \"bpm\": %.2f, \"score\": %.4f, \"fft_norm\": %.4f, \"autocorr_norm\": %.4f, "
                            "\"selected\": %s }%s\n",
                            (double)c.bpm, (double)c.score, (double)c.fft_norm, (double)c.autocorr_norm,
                            c.selected ? "true" : "false", i + 1 == res.n_tempogram_candidates ? "" : ",");
            }
            std::printf("  ],\n");
        }
        std::printf("  \"processing_time_ms\": %.2f\n", (double)res.processing_time_ms);
        std::printf("}\n");
    } else {
        std::printf("Analysis Results:\n");
        std::printf("  BPM: %.2f (confidence: %.2f)\n", (double)res.bpm, (double)conf.bpm_confidence);
        std::printf("  Key: %s (confidence: %.2f, clarity: %.2f)\n", key.c_str(), (double)conf.key_confidence,
                    (double)res.key_clarity);
        std::printf("  Grid stability: %.2f\n", (double)res.grid_stability);
        std::printf("  Processing time: %.2f ms\n", (double)res.processing_time_ms);
    }
    sdsp_result_free(&res);
    return 0;
}
