// Host-only harness for stratum-dsp_amd/csrc/batch_sched.hpp (the chunk queue of
// sdsp_analyze_batch), driven with fake devices.  Each fake device has two "HBM" slots; stage()
// copies the chunk's track ids into a slot, analyze() reads the slot back and writes every track's
// result into its own output position.  Checks: every track analysed exactly once, in its own
// slot, by a device that held it; failures reported per chunk; chunks of a device whose copier
// dies are taken over by the others.  Usage: batch_sched_test <scenario> <seed>.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../stratum-dsp_amd/csrc/batch_sched.hpp"

int main(int argc, char** argv) {
    const std::string scen = argc > 1 ? argv[1] : "basic";
    const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1u;
    std::mt19937 rng(seed);
    const uint64_t n = 997;
    std::vector<uint64_t> lens(n);
    for (auto& l : lens) l = 1 + rng() % 50;
    lens[5] = 0;  // an empty track travels like any other
    const std::vector<uint64_t> cb = sdsp::plan_chunks(lens.data(), n, 37, 600);
    // chunks: contiguous, whole, bounded
    if (cb.front() != 0 || cb.back() != n) return 10;
    for (size_t c = 0; c + 1 < cb.size(); c++) {
        if (cb[c + 1] <= cb[c] || cb[c + 1] - cb[c] > 37) return 11;
        uint64_t tot = 0;
        for (uint64_t i = cb[c]; i < cb[c + 1]; i++) tot += lens[i];
        if (tot > 600 && cb[c + 1] - cb[c] > 1) return 12;
    }
    const size_t n_chunks = cb.size() - 1;
    const int ndev = scen == "single" ? 1 : 3;
    std::vector<std::vector<std::vector<int64_t>>> slots(ndev, std::vector<std::vector<int64_t>>(2));
    std::vector<int> hits(n, 0), out_id(n, -1), out_dev(n, -1);
    std::vector<int> failed_chunk(n_chunks, 0);
    std::mutex mu;
    std::vector<sdsp::ChunkDevice> devs(ndev);
    for (int d = 0; d < ndev; d++) {
        devs[d].stage = [&, d](int s, size_t c) {
            if (scen == "copier_dies" && d == 1) throw std::runtime_error("stage failed");
            if (scen == "all_copiers_die") throw std::runtime_error("stage failed");
            if (scen == "copier_throws_int" && d == 1) throw 42;  // not a std::exception
            thread_local std::mt19937 trng(seed * 7919u + (unsigned)d);
            std::this_thread::sleep_for(std::chrono::microseconds(trng() % 300));
            auto& sl = slots[d][s];
            sl.clear();
            for (uint64_t i = cb[c]; i < cb[c + 1]; i++) sl.push_back((int64_t)i);
        };
        devs[d].analyze = [&, d](int s, size_t c) {
            // every fourth chunk fails on whichever device takes it (which device takes a chunk
            // depends on timing; tying the failure to one device let a loaded host schedule it none)
            if (scen == "analyze_fails" && c % 4 == 1) throw std::runtime_error("analysis failed");
            if (scen == "analyze_throws_int" && c % 4 == 1) throw 7;  // not a std::exception
            std::this_thread::sleep_for(std::chrono::microseconds(d == 0 ? 900 : 200));
            const auto& sl = slots[d][s];
            if (sl.size() != cb[c + 1] - cb[c]) throw std::logic_error("slot holds another chunk");
            std::lock_guard<std::mutex> lk(mu);
            for (size_t k = 0; k < sl.size(); k++) {
                const uint64_t i = cb[c] + k;
                if (sl[k] != (int64_t)i) {
                    std::fprintf(stderr, "slot mismatch\n");
                    std::exit(20);
                }
                hits[i]++;
                out_id[i] = (int)sl[k];
                out_dev[i] = d;
            }
        };
        devs[d].drain = [] {};
    }
    const size_t nf = sdsp::run_chunked(n_chunks, devs, [&](size_t c, const std::string&) { failed_chunk[c]++; });
    size_t expect_fail = 0;
    for (size_t c = 0; c < n_chunks; c++) {
        for (uint64_t i = cb[c]; i < cb[c + 1]; i++) {
            if (failed_chunk[c]) {
                if (hits[i] != 0) return 30;  // a failed chunk's tracks are not also analysed
            } else if (hits[i] != 1 || out_id[i] != (int)i) {
                std::fprintf(stderr, "track %llu hits %d\n", (unsigned long long)i, hits[i]);
                return 31;
            }
        }
        if (failed_chunk[c] > 1) return 32;
        expect_fail += failed_chunk[c];
    }
    if (nf != expect_fail) return 33;
    if (scen == "basic" || scen == "single" || scen == "copier_dies" || scen == "copier_throws_int") {
        if (nf != 0) return 34;
    }
    if (scen == "copier_dies" || scen == "copier_throws_int")
        for (uint64_t i = 0; i < n; i++)
            if (out_dev[i] == 1) return 35;  // device 1 never held a chunk
    if ((scen == "analyze_fails" || scen == "analyze_throws_int") && nf != (n_chunks + 2) / 4) return 36;
    if (scen == "all_copiers_die" && nf != n_chunks) return 37;
    int used = 0;
    for (int d = 0; d < ndev; d++)
        for (uint64_t i = 0; i < n; i++)
            if (out_dev[i] == d) {
                used++;
                break;
            }
    std::printf("ok %s chunks=%zu failed=%zu devices_used=%d\n", scen.c_str(), n_chunks, nf, used);
    return 0;
}
