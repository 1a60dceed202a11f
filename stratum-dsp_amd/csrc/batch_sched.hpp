// batch_sched.hpp — the chunk queue behind sdsp_analyze_batch (host buffers, one or more GPUs).
//
// Replaces the caller-side fan-out of the reference (examples/analyze_batch.rs:239-268: rayon,
// one track per task): the batch is cut into chunks of whole tracks, and one worker per device
// pulls chunks from a shared counter, so escalation-heavy chunks do not leave other GPUs idle
// (SURVEY §8e).  Per device a copier thread stages the next chunk into the second of two slots
// while the worker analyses the current one.
//
// This header is host-only (no HIP): the GPU side supplies the three callbacks, and
// tests/test_batch_sched.py drives the same code with fake devices.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace sdsp {

// Chunk boundaries cb[0] = 0 < cb[1] < ... < cb[n_chunks] = n: whole tracks, at most
// max_tracks tracks and (unless a single track is larger) max_samples samples per chunk.
inline std::vector<uint64_t> plan_chunks(const uint64_t* lens, uint64_t n, uint64_t max_tracks, uint64_t max_samples) {
    std::vector<uint64_t> cb(1, 0);
    if (n == 0) return cb;
    max_tracks = std::max<uint64_t>(max_tracks, 1);
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (i > cb.back() && (i - cb.back() >= max_tracks || acc + lens[i] > max_samples)) {
            cb.push_back(i);
            acc = 0;
        }
        acc += lens[i];
    }
    cb.push_back(n);
    return cb;
}

// Per-device callbacks.  stage() runs on the device's copier thread, analyze() and drain() on its
// worker thread; any of them may throw.  After analyze() throws, drain() must return only once the
// device no longer reads either slot (the slot is then reused).
struct ChunkDevice {
    std::function<void(int slot, size_t chunk)> stage;
    std::function<void(int slot, size_t chunk)> analyze;
    std::function<void()> drain;
};

// Runs every chunk exactly once on some device.  fail(chunk, what) is called for each chunk whose
// staging or analysis threw (its tracks keep an error status); chunks never staged because a
// copier failed are re-queued to the devices that still work, and fail()ed only if none is left.
// Returns the number of failed chunks.
inline size_t run_chunked(size_t n_chunks, std::vector<ChunkDevice>& devs,
                          const std::function<void(size_t chunk, const std::string& what)>& fail) {
    std::atomic<size_t> next{0};
    std::atomic<size_t> n_failed{0};
    std::mutex fmu;  // serialises fail() and the orphan list
    std::vector<size_t> orphans;  // chunks taken by a copier that died before staging them
    auto fail_one = [&](size_t c, const std::string& what) {
        std::lock_guard<std::mutex> lk(fmu);
        fail(c, what);
        n_failed++;
    };
    auto device_worker = [&](size_t k) {
        ChunkDevice& dv = devs[k];
        std::mutex mu;
        std::condition_variable cv;
        long ready[2] = {-1, -1};  // chunk staged in slot s, -1 = free
        bool done = false;
        auto copier = [&]() {
            int s = 0;
            for (;;) {
                const size_t c = next++;
                if (c >= n_chunks) break;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return ready[s] < 0; });
                }
                bool staged = true;
                try {
                    dv.stage(s, c);
                } catch (...) {  // any exception type: a std::thread must not let one escape
                    staged = false;
                }
                if (!staged) {
                    // this device cannot stage: hand the chunk back and stop copying for it
                    std::lock_guard<std::mutex> lk(fmu);
                    orphans.push_back(c);
                    break;
                }
                {
                    std::lock_guard<std::mutex> lk(mu);
                    ready[s] = (long)c;
                }
                cv.notify_all();
                s ^= 1;
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                done = true;
            }
            cv.notify_all();
        };
        std::thread cp(copier);
        int s = 0;
        for (;;) {
            long c;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return ready[s] >= 0 || (done && ready[0] < 0 && ready[1] < 0); });
                if (ready[s] < 0) break;  // copier finished and nothing staged
                c = ready[s];
            }
            std::string why;
            bool ok = true;
            try {
                dv.analyze(s, (size_t)c);
            } catch (const std::exception& e) {
                ok = false;
                why = e.what();
            } catch (...) {
                ok = false;
                why = "unknown exception";
            }
            if (!ok) {
                fail_one((size_t)c, why);
                try {
                    if (dv.drain) dv.drain();
                } catch (...) {
                }
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                ready[s] = -1;
            }
            cv.notify_all();
            s ^= 1;
        }
        cp.join();
    };
    if (devs.size() == 1) {
        device_worker(0);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 0; k < devs.size(); k++) th.emplace_back(device_worker, k);
        for (auto& t : th) t.join();
    }
    // chunks a dying copier gave back, and chunks no copier took because every copier died:
    // staged and run serially on the first device that takes them; failed if none can
    for (size_t c = std::min(next.load(), n_chunks); c < n_chunks; c++) orphans.push_back(c);
    std::sort(orphans.begin(), orphans.end());
    for (size_t c : orphans) {
        bool ok = false;
        std::string why = "no device could stage the chunk";
        for (auto& dv : devs) {
            try {
                dv.stage(0, c);
            } catch (const std::exception& e) {
                why = e.what();
                continue;
            } catch (...) {
                why = "unknown exception";
                continue;
            }
            bool threw = false;
            try {
                dv.analyze(0, c);
                ok = true;
            } catch (const std::exception& e) {
                why = e.what();
                threw = true;
            } catch (...) {
                why = "unknown exception";
                threw = true;
            }
            if (threw) {
                try {
                    if (dv.drain) dv.drain();
                } catch (...) {
                }
            }
            break;
        }
        if (!ok) fail_one(c, why);
    }
    return n_failed.load();
}

}  // namespace sdsp
