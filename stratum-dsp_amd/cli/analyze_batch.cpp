// analyze_batch — batch front-end with the reference example's interface and output
// (examples/analyze_batch.rs): files are decoded on host worker threads (--jobs, default
// CPU threads - 1), then analysed on the GPUs as one batch per sample rate through
// sdsp_analyze_batch (sharded over --devices, default every visible GPU), each result scored
// with compute_confidence, printed in input order as text lines or JSONL, with the same
// summary on stderr.
//
//   analyze_batch [--jobs N] [--devices MASK] [--json] <file1> <file2> ...
#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <thread>

#include "cli_common.hpp"

using namespace sdsp_cli;

namespace {

struct Item {
    std::string path;
    std::vector<float> samples;
    uint32_t sr = 0;
    bool decoded = false;
    std::string error;
    bool ok = false;
    float bpm = 0, bpm_conf = 0, key_conf = 0, ms = 0;
    std::string key;
    int8_t tr[4] = {-1, -1, -1, -1};
};

// percentile as the example computes it: sort, index round((len-1) * p)
float percentile(std::vector<float> xs, float p) {
    std::sort(xs.begin(), xs.end());
    const float q = p < 0.0f ? 0.0f : p > 1.0f ? 1.0f : p;
    size_t idx = (size_t)std::roundf((float)(xs.size() - 1) * q);  // f32::round: half away from zero
    if (idx >= xs.size()) idx = xs.size() - 1;
    return xs[idx];
}

}  // namespace

int main(int argc, char** argv) {
    Args a(argv + 1, argv + argc);
    bool json = false;
    uint64_t jobs = 0;
    uint32_t devices = 0;
    std::vector<std::string> paths;
    for (size_t i = 0; i < a.size(); i++) {
        const std::string& s = a[i];
        if (s == "--json") {
            json = true;
        } else if (s == "--jobs" || s == "--devices") {
            uint64_t v;
            if (i + 1 >= a.size() || !parse_usize_str(a[i + 1], &v)) {
                std::fprintf(stderr, "Error: %s requires a value\n", s.c_str());
                return 1;
            }
            if (s == "--jobs")
                jobs = std::max<uint64_t>(1, v);
            else
                devices = (uint32_t)v;
            i++;
        } else if (s == "--help" || s == "-h") {
            std::fprintf(stderr,
                         "Usage: analyze_batch [--jobs N] [--devices MASK] [--json] <file1> <file2> ...\n\n"
                         "--jobs N        Decode workers (default: CPU-1)\n"
                         "--devices MASK  GPU bitmask (default: all visible GPUs)\n"
                         "--json          Emit one JSON object per line (JSONL)\n");
            return 0;
        } else {
            paths.push_back(s);
        }
    }
    if (paths.empty()) {
        std::fprintf(stderr, "ERROR: Provide at least one audio file path. Use --help for usage.\n");
        return 2;
    }
    if (jobs == 0) {
        const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
        jobs = std::max<uint64_t>(1, hc - 1);
    }
    if (devices == 0) {
        const int nd = sdsp_device_count();
        devices = nd >= 32 ? 0xffffffffu : nd > 0 ? ((1u << nd) - 1) : 1u;
    }
    std::fprintf(stderr, "Batch: %zu files, jobs=%llu\n", paths.size(), (unsigned long long)jobs);
    const auto t0 = std::chrono::steady_clock::now();

    std::vector<Item> items(paths.size());
    std::atomic<size_t> next{0};
    auto worker = [&]() {
        for (size_t i; (i = next++) < items.size();) {
            Item& it = items[i];
            it.path = paths[i];
            float* p = nullptr;
            uint64_t n = 0;
            char err[512];
            if (sdsp_decode_audio_file(it.path.c_str(), &p, &n, &it.sr, err, sizeof err) != 0) {
                it.error = std::string("decode failed: ") + err;
                continue;
            }
            it.samples.assign(p, p + n);
            sdsp_free_samples(p);
            it.decoded = true;
        }
    };
    std::vector<std::thread> pool;
    for (uint64_t j = 0; j < std::min<uint64_t>(jobs, items.size()); j++) pool.emplace_back(worker);
    for (auto& t : pool) t.join();

    sdsp_config cfg;
    sdsp_config_default(&cfg);
    std::map<uint32_t, std::vector<size_t>> by_sr;
    for (size_t i = 0; i < items.size(); i++)
        if (items[i].decoded) by_sr[items[i].sr].push_back(i);
    for (auto& kv : by_sr) {
        const std::vector<size_t>& idx = kv.second;
        std::vector<const float*> ptrs;
        std::vector<uint64_t> lens;
        for (size_t i : idx) {
            ptrs.push_back(items[i].samples.data());
            lens.push_back(items[i].samples.size());
        }
        std::vector<sdsp_result> outs(idx.size());
        // a non-OK return means some chunk failed; every track's own status says which (tracks the
        // library did not analyse carry an error status), so each result is read and freed
        (void)sdsp_analyze_batch(ptrs.data(), lens.data(), idx.size(), kv.first, &cfg, devices, outs.data());
        for (size_t k = 0; k < idx.size(); k++) {
            Item& it = items[idx[k]];
            const sdsp_result& r = outs[k];
            if (r.status != 0) {
                it.error = std::string("analysis failed: ") + r.error_message;
            } else {
                sdsp_confidence c;
                sdsp_compute_confidence(&r, &c);
                it.ok = true;
                it.bpm = r.bpm;
                it.bpm_conf = c.bpm_confidence;
                it.key = key_name(r);
                it.key_conf = c.key_confidence;
                it.ms = r.processing_time_ms;
                it.tr[0] = r.tempogram_multi_res_triggered;
                it.tr[1] = r.tempogram_multi_res_used;
                it.tr[2] = r.tempogram_percussive_triggered;
                it.tr[3] = r.tempogram_percussive_used;
            }
            sdsp_result_free(&outs[k]);
        }
    }

    for (size_t i = 0; i < items.size(); i++) {
        const Item& o = items[i];
        if (json) {
            if (o.ok)
                std::printf("{\"file\":%s,\"bpm\":%.2f,\"bpm_confidence\":%.4f,\"key\":%s,\"key_confidence\":%.4f,"
                            "\"processing_time_ms\":%.2f,\"tempogram_multi_res_triggered\":%s,"
                            "\"tempogram_multi_res_used\":%s,\"tempogram_percussive_triggered\":%s,"
                            "\"tempogram_percussive_used\":%s}\n",
                            json_str(o.path).c_str(), (double)o.bpm, (double)o.bpm_conf, json_str(o.key).c_str(),
                            (double)o.key_conf, (double)o.ms, tri(o.tr[0]), tri(o.tr[1]), tri(o.tr[2]), tri(o.tr[3]));
            else
                std::printf("{\"file\":%s,\"error\":%s}\n", json_str(o.path).c_str(),
                            json_str(o.error.empty() ? "unknown error" : o.error).c_str());
        } else {
            if (o.ok)
                std::printf("[%zu/%zu] %s: BPM=%.2f (conf=%.3f) Key=%s (conf=%.3f) time=%.2fms\n", i + 1, items.size(),
                            o.path.c_str(), (double)o.bpm, (double)o.bpm_conf, o.key.c_str(), (double)o.key_conf,
                            (double)o.ms);
            else
                std::printf("[%zu/%zu] %s: ERROR: %s\n", i + 1, items.size(), o.path.c_str(),
                            o.error.empty() ? "unknown error" : o.error.c_str());
        }
    }
    std::vector<float> ok_times;
    for (const Item& o : items)
        if (o.ok) ok_times.push_back(o.ms);
    const double wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "Done: ok=%zu/%zu wall=%.0fms\n", ok_times.size(), items.size(), wall_ms);
    if (!ok_times.empty()) {
        float sum = 0.0f;
        for (float t : ok_times) sum += t;
        const float mean = sum / (float)ok_times.size();
        float mn = INFINITY, mx = 0.0f;
        for (float t : ok_times) {
            mn = std::min(mn, t);
            mx = std::max(mx, t);
        }
        std::fprintf(stderr, "processing_time_ms: mean=%.2f p50=%.2f p90=%.2f min=%.2f max=%.2f\n", (double)mean,
                     (double)percentile(ok_times, 0.50f), (double)percentile(ok_times, 0.90f), (double)mn, (double)mx);
    }
    return 0;
}
