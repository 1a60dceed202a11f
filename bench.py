#!/usr/bin/env python3
"""Throughput benchmark: full default-config analyze_audio() on synthetic 3-min 44.1 kHz tracks.

Metric (BASELINE.json): tracks/sec of full analyze_audio() at 1/2/4/8 MI355X.  One "step" is one
pass of the whole pipeline over one batch of `--tracks` tracks per GPU (BASELINE config 2: 1024
per GPU; config 3 = 8 GPUs x 1024).  Tracks are generated on the device before the timed region
(inputs resident in HBM); every step re-runs everything, results are copied back to the host.

Multi-GPU: one process per GPU (torch.distributed.run), tracks sharded with no data-path
collective (`scaling: weak`); a gloo (CPU) process group provides the barrier and the max over
ranks.  The engine's own HIP runtime is loaded before torch so no second GPU runtime is touched.

Also reported: the dominant STFT kernel's HBM roofline (algorithmic bytes / HIP-event kernel time
vs 8 TB/s) and the CPU restatement (oracle) timed on this box's host cores on a bounded sample.
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "stratum-dsp_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import sdsp  # noqa: E402  (loads libstratum_hip.so first)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


class Engine:
    """The HIP engine through its C ABI (libstratum_hip.so): tracks generated and kept in HBM."""

    def __init__(self, dev):
        sdsp.lib()
        self.dev = dev

    def generate(self, n, L, sr, seed0, bpm_mode):
        buf = sdsp.DeviceBuffer(n * L, device=self.dev)
        sdsp.generate_synthetic(buf.ptr, n, L, sr, seed0=seed0, bpm_mode=bpm_mode, device=self.dev)
        return buf

    def analyze(self, buf, offs, lens, sr):
        return sdsp.analyze_batch_device(buf.ptr, offs, lens, sr, device=self.dev, raw=True)

    def stage_times(self):
        return sdsp.stage_times(self.dev)

    def synchronize(self):
        sdsp.synchronize(self.dev)


class DryEngine:
    """--dry-run: rehearses the launcher / sharding / timing / reporting logic on the CPU (the
    multi-process tests drive it with gloo); it measures nothing."""

    class _Res:
        def __init__(self, n):
            self.status = [0] * n

        def free(self):
            pass

    def __init__(self, dev):
        self.dev = dev

    def generate(self, n, L, sr, seed0, bpm_mode):
        return {"n": n, "seed0": seed0}

    def analyze(self, buf, offs, lens, sr):
        time.sleep(0.001 * len(lens))
        return DryEngine._Res(len(lens))

    def stage_times(self):
        return {k: 0.0 for k in ("stft2048_ms", "stft8192_ms", "stft2048_bytes", "stft8192_bytes", "total_ms")} | {
            "stft2048_launches": 0, "stft8192_launches": 0}

    def synchronize(self):
        pass


def shard_seed0(rank, tracks_per_rank):
    """First synthetic seed of this rank: ranks own disjoint, contiguous track ranges."""
    return rank * tracks_per_rank


def max_over_ranks(dt, tdist):
    """The job's time = the slowest rank's (weak scaling, no data-path collective)."""
    if tdist is None:
        return dt
    import torch

    t = torch.tensor([dt], dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tracks", type=int, default=1024, help="tracks per GPU per step")
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, os.cpu_count())")
    ap.add_argument("--cpu-tracks", type=int, default=0, help="0 = 2 per thread")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bpm-mode", type=int, default=0, help="1 = config-5 escalation-heavy BPM mix")
    ap.add_argument("--dry-run", action="store_true", help="host-logic rehearsal without a GPU (tests)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    eng = (DryEngine if args.dry_run else Engine)(local)
    tdist = None
    if world > 1:
        import torch.distributed as tdist

        tdist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if tdist is not None:
            tdist.barrier()

    sr = 44100
    n = args.tracks
    L = int(args.seconds * sr)
    buf = eng.generate(n, L, sr, shard_seed0(rank, n), args.bpm_mode)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, dtype=np.uint64)

    # results stay native (C-ABI structs, as a Rust/C caller receives them); the parity sample
    # below converts the tracks it checks
    for _ in range(args.warmup):
        eng.analyze(buf, offs, lens, sr).free()
    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    stft = {"ms8": 0.0, "b8": 0.0, "l8": 0, "ms2": 0.0, "b2": 0.0, "l2": 0}
    res = None
    for _ in range(args.steps):
        if res is not None:
            res.free()
        res = eng.analyze(buf, offs, lens, sr)
        st = eng.stage_times()
        stft["ms8"] += st["stft8192_ms"]
        stft["b8"] += st["stft8192_bytes"]
        stft["l8"] += st["stft8192_launches"]
        stft["ms2"] += st["stft2048_ms"]
        stft["b2"] += st["stft2048_bytes"]
        stft["l2"] += st["stft2048_launches"]
    eng.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0, tdist)
    n_err = sum(1 for st in res.status if st != 0)
    total_tracks = n * world * args.steps
    value = total_tracks / dt
    stages = eng.stage_times()
    # roofline of the dominant STFT kernel (k_stft_mag<8192>): algorithmic bytes per launch
    # (4*N_in + 4*F*(nfft/2+1)) / average launch time (HIP events on the engine stream)
    l8 = max(stft["l8"], 1)
    bytes_per_launch = stft["b8"] / l8
    ms_per_launch = stft["ms8"] / l8
    achieved = bytes_per_launch / (ms_per_launch * 1e-3) / 1e9 if ms_per_launch > 0 else 0.0
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_stft8192.json")
    if os.path.exists(pmc_path):
        # rocprofv3 PMC passes (profiles/README.md): measured HBM bytes / algorithmic bytes for
        # this kernel; scales to the per-launch traffic of whatever batch this run used
        with open(pmc_path) as f:
            ratio = json.load(f).get("hbm_over_algorithmic")
        if ratio is not None:
            traffic = round(ratio * bytes_per_launch)
    roofline = {
        "bound": "hbm",
        "kernel": "k_stft_mag<8192> (key STFT, 8192/512)",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "bytes_per_launch": bytes_per_launch,
        "ms_per_launch": ms_per_launch,
        "stft2048_GBps": round(stft["b2"] / (stft["ms2"] * 1e-3) / 1e9, 2) if stft["ms2"] > 0 else None,
        "stft_stage_GBps": round((stft["b2"] + stft["b8"]) / ((stft["ms2"] + stft["ms8"]) * 1e-3) / 1e9, 2)
        if (stft["ms2"] + stft["ms8"]) > 0 else None,
    }

    cpu = None
    parity = None
    extras = {}
    if not args.dry_run:
        # fraction of this rank's tracks whose base estimate escalated to multi-resolution
        # (src/lib.rs:410-459; BASELINE.md asks for the escalation rate beside the throughput)
        extras["escalation_rate"] = round(res.count("tempogram_multi_res_triggered") / max(n, 1), 4)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run:
        cpu, parity = cpu_baseline(buf, res, n, L, sr, args)
        extras["sine_30s"] = sine_30s(sr)

    if rank == 0:
        out = {
            "metric": "tracks/sec full analyze_audio(), 3-min 44.1 kHz mono, at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "tracks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded on-device generator: kick/hat/triad/diatonic line, 3-min 44.1 kHz mono)"
            + (" [DRY RUN: no GPU, not a measurement]" if args.dry_run else ""),
            "config": {
                "workload": f"batch of {n} synthetic {args.seconds:g}-s 44.1 kHz mono tracks per GPU, "
                            "AnalysisConfig::default(), full BPM + key + beat grid",
                "tracks_per_gpu": n,
                "seconds_per_track": args.seconds,
                "sample_rate": sr,
                "bpm_mode": args.bpm_mode,
                "parallelism": f"track-sharded x{world} (no collectives)",
            },
            "errors": n_err,
            "stage_ms_last_step": {k: round(v, 3) for k, v in stages.items() if k.endswith("_ms")},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity_sample": parity,
            **extras,
        }
        print(json.dumps(out), flush=True)
    if tdist is not None:
        tdist.destroy_process_group()


def cpu_baseline(buf, res, n, L, sr, args):
    """The oracle (C++ restatement, single-threaded per track, one track per thread as
    examples/analyze_batch.rs:239-268 does with rayon) on a bounded sample of the same tracks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import parity

    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    k = min(n, args.cpu_tracks or 2 * threads)
    xs = [buf.to_host(i * L, L) for i in range(k)]
    oracle.lib()

    def one(x):
        return oracle.analyze(x, sr)

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(one, xs))
    dt = time.perf_counter() - t0
    match = sum(1 for i, (st, ref) in enumerate(outs) if st == 0 and not parity.diff_results(res[i], ref))
    exact = sum(1 for i, (st, ref) in enumerate(outs) if st == 0 and parity.exact_fraction(res[i], ref) == 1.0)
    cpu = {
        "value": round(k / dt, 4),
        "unit": "tracks/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{k} of the benchmark's own {args.seconds:g}-s tracks, one track per thread, "
                  f"{dt:.1f} s wall ({dt * threads:.0f} thread-s); C++ restatement -O3, FFT per sdsp_fft_spec.h",
    }
    # one thread, the same tracks (report 1 thread and all cores)
    k1 = min(k, 2)
    t0 = time.perf_counter()
    for x in xs[:k1]:
        one(x)
    cpu["value_1thread"] = round(k1 / (time.perf_counter() - t0), 4)
    par = {"checked": k, "within_tolerance": match, "bit_exact": exact}
    return cpu, par


def sine_30s(sr):
    """The reference's own Criterion workload (benches/audio_analysis_bench.rs:25-29,410-423):
    one 30-s 440 Hz sine at amplitude 0.5, one analyze_audio call.  GPU: host buffer in, results
    out (H2D included), median of 5 calls after one warmup; CPU: the oracle on one thread.  The
    reference publishes ~203-208 ms for it on its author's machine."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    i = np.arange(sr * 30, dtype=np.float32)
    f32 = np.float32
    x = (np.sin(i * f32(440.0) * f32(2.0) * f32(np.pi) / f32(sr)) * f32(0.5)).astype(np.float32)  # f32 ops, Rust order
    sdsp.analyze_audio(x, sr)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        sdsp.analyze_audio(x, sr)
        ts.append((time.perf_counter() - t0) * 1e3)
    t0 = time.perf_counter()
    oracle.analyze(x, sr)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    return {"gpu_ms": round(sorted(ts)[2], 3), "cpu_port_1thread_ms": round(cpu_ms, 1),
            "reference_published_ms": "203-208 (author's machine, Criterion)"}


if __name__ == "__main__":
    main()
