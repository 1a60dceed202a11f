#!/usr/bin/env python3
"""Key parity at the benchmark's own scale under the default key path's block-folded HPCP
energies (k_mask_rp / k_hpcp_band): the GPU engine against the oracle on every track
of a benchmark shard, not a sample.

    python tools/key_scale_check.py [--n 1024] [--sets config2,config5] [--threads 0] [--out FILE]

Sets (the tracks bench.py generates, on the device, with the same seeds):
  config2  seeds 0..n-1, 3-min 44.1 kHz, the bench's default mix (bpm_mode 0), full analysis;
  config5  seeds 0..n-1, 3-min, the escalation-heavy BPM mix of BASELINE config 5 (bpm_mode 1),
           analysed in FULL (key included), so the key path runs on the config-5 tracks too.
Per set: key equal count, tracks within the north-star tolerance, tracks bit-exact in every field
but the two re-associated ones, strict bit-exact count, worst |diff| of key_confidence /
key_clarity, and the tracks whose key differs (if any).  The oracle runs on the host's CPU share
(OMP_NUM_THREADS, one track per thread); a progress line is printed every 64 tracks.
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stratum-dsp_amd", "python"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import parity  # noqa: E402
import sdsp  # noqa: E402

SETS = {"config2": 0, "config5": 1}


def run_set(name, n, threads, sr=44100, seconds=180.0):
    length = int(seconds * sr)
    buf = sdsp.DeviceBuffer(n * length)
    sdsp.generate_synthetic(buf.ptr, n, length, sr, seed0=0, bpm_mode=SETS[name])
    offs = np.arange(n, dtype=np.uint64) * np.uint64(length)
    lens = np.full(n, length, dtype=np.uint64)
    t0 = time.time()
    res = sdsp.analyze_batch_device(buf.ptr, offs, lens, sr, raw=True)
    gpu_s = time.time() - t0
    st = sdsp.stage_times()
    nb = sdsp.last_key_near(n)
    near = [int(i) for i in np.nonzero(nb)[0]]
    why = {name: int(((nb & bit) != 0).sum()) for name, bit in (("argmax", 1), ("gate", 2), ("final", 4), ("wsum", 8), ("range", 16))}
    out = {"set": name, "tracks": n, "bpm_mode": SETS[name], "seeds": [0, n - 1], "gpu_s": round(gpu_s, 2),
           "gpu_errors": sum(1 for s in res.status if s != 0), "key_equal": 0, "within_tol": 0,
           "bit_exact_except_key_energy": 0, "bit_exact_strict": 0, "max_key_confidence_diff": 0.0,
           "max_key_clarity_diff": 0.0, "escalated": res.count("tempogram_multi_res_triggered"),
           "key_reruns": int(st.get("key_reruns", 0)), "rerun_ms": round(float(st.get("rerun_ms", 0.0)), 1),
           "near_reasons": why, "near_tracks": near, "key_mismatch": [], "tolerance_fail": []}

    def one(i):
        x = buf.to_host(int(offs[i]), length)
        return i, oracle.analyze(x, sr)

    oracle.lib()
    t0 = time.time()
    done = 0
    with cf.ThreadPoolExecutor(threads) as ex:
        for i, (st, ref) in ex.map(one, range(n)):
            r = res[i]
            done += 1
            if st != 0 or isinstance(r, Exception):
                out["tolerance_fail"].append([i, "error", str(r), st])
                continue
            out["key_equal"] += int(r["key"] == ref["key"])
            if r["key"] != ref["key"]:
                out["key_mismatch"].append([i, r["key"], ref["key"], r["key_clarity"], ref["key_clarity"]])
            d = parity.diff_results(r, ref)
            out["within_tol"] += int(not d)
            if d:
                out["tolerance_fail"].append([i, d])
            g, e = parity.result_digest(r), parity.result_digest(ref)
            out["bit_exact_except_key_energy"] += int(all(g[k] == e[k] for k in g if k not in parity.KEY_ENERGY_FIELDS))
            out["bit_exact_strict"] += int(g == e)
            out["max_key_confidence_diff"] = max(out["max_key_confidence_diff"],
                                                 abs(float(r["key_confidence"]) - float(ref["key_confidence"])))
            out["max_key_clarity_diff"] = max(out["max_key_clarity_diff"],
                                              abs(float(r["key_clarity"]) - float(ref["key_clarity"])))
            if done % 64 == 0:
                print(f"# {name}: {done}/{n} tracks, {time.time() - t0:.0f} s, key equal {out['key_equal']}",
                      flush=True)
    out["oracle_s"] = round(time.time() - t0, 1)
    out["oracle_threads"] = threads
    res.free()
    buf.free()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--sets", default="config2,config5")
    ap.add_argument("--threads", type=int, default=0, help="0 = the box's CPU share (OMP_NUM_THREADS)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    threads = a.threads or int(os.environ.get("OMP_NUM_THREADS", "") or os.cpu_count() or 1)
    lines = []
    for name in a.sets.split(","):
        r = run_set(name, a.n, threads)
        print(json.dumps(r), flush=True)
        lines.append(r)
    if a.out:
        with open(a.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
