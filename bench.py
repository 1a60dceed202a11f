#!/usr/bin/env python3
"""Throughput benchmark: full default-config analyze_audio() on synthetic 3-min 44.1 kHz tracks.

Metric (BASELINE.json): tracks/sec of full analyze_audio() at 1/2/4/8 MI355X.  One "step" is one
pass of the whole pipeline over one batch of `--tracks` tracks per GPU (BASELINE config 2: 1024
per GPU; config 3 = 8 GPUs x 1024).  Tracks are generated on the device before the timed region
(inputs resident in HBM); every step re-runs everything, results are copied back to the host.

Multi-GPU: one process per GPU, tracks sharded with no data-path collective (`scaling: weak`); a
gloo (CPU) process group provides the barrier and the max over ranks.  Under torch.distributed.run
the ranks come from the environment; `python bench.py --gpus N` without it spawns the N rank
processes itself (before anything touches a GPU) and exits with their status.  The engine's own
HIP runtime is loaded before torch so no second GPU runtime is touched.

Workloads (BASELINE.json configs): `config2` (default) 1024 x 3-min tracks per GPU, full analysis;
`mixed` (config 4) lengths uniform on whole seconds in [30, 600]; `bpm-only` (config 5) 4096
tracks per GPU with an escalation-heavy BPM mix, stages a1-a19 only.

Also reported: the dominant STFT kernel's HBM roofline (algorithmic bytes / HIP-event kernel time
vs 8 TB/s) and the CPU restatement (oracle) timed on this box's host cores on a bounded sample.
"""
import argparse
import concurrent.futures as cf
import json
import os
import re
import socket
import subprocess
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

    def generate(self, lens, sr, seed0, bpm_mode):
        """Track i (seed seed0 + i) of lens[i] samples at offs[i] of one HBM buffer."""
        lens = np.asarray(lens, dtype=np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        buf = sdsp.DeviceBuffer(int(lens.sum()), device=self.dev)
        if np.all(lens == lens[0]):
            sdsp.generate_synthetic(buf.ptr, len(lens), int(lens[0]), sr, seed0=seed0, bpm_mode=bpm_mode, device=self.dev)
        else:
            for i, (o, ln) in enumerate(zip(offs, lens)):
                sdsp.generate_synthetic(buf.ptr + 4 * int(o), 1, int(ln), sr, seed0=seed0 + i, bpm_mode=bpm_mode,
                                        device=self.dev)
        return buf, offs

    def analyze(self, buf, offs, lens, sr, stages=0):
        return sdsp.analyze_batch_device(buf.ptr, offs, lens, sr, device=self.dev, raw=True, stages=stages)

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

    def generate(self, lens, sr, seed0, bpm_mode):
        lens = np.asarray(lens, dtype=np.uint64)
        return {"n": len(lens), "seed0": seed0}, np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)

    def analyze(self, buf, offs, lens, sr, stages=0):
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


WORKLOADS = {
    # name: (BASELINE config, default tracks per GPU, synthetic BPM mix, stages)
    "config2": (2, 1024, 0, 0),
    "mixed": (4, 1024, 0, 0),
    "bpm-only": (5, 4096, 1, 1),
}


def track_lengths(workload, n, seconds, sr, seed0):
    """Per-track sample counts.  mixed (config 4): whole seconds uniform on [30, 600], seeded by
    the rank's first track so ranks draw disjoint, reproducible lengths."""
    if workload == "mixed":
        rng = np.random.default_rng(0x5EED0000 + seed0)
        return (rng.integers(30, 601, size=n) * sr).astype(np.uint64)
    return np.full(n, int(seconds * sr), dtype=np.uint64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`bench.py --gpus N` outside torch.distributed.run: start N fresh rank processes (rank r on
    GPU r) with the torchrun environment and wait for them.  This process touches no GPU; rank 0
    prints the JSON line.  Returns the worst exit status."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e))
    # poll: a rank that dies before the barrier would leave its siblings blocked in gloo, so the
    # first non-zero exit ends the others and is returned
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="config2")
    ap.add_argument("--tracks", type=int, default=0, help="tracks per GPU per step (0 = the workload's)")
    ap.add_argument("--seconds", type=float, default=180.0, help="track length (config2 / bpm-only)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every host core this process may use (its affinity set, capped by the box's CPU share)")
    ap.add_argument("--cpu-tracks", type=int, default=0, help="0 = 2 per thread")
    ap.add_argument("--cpu-1thread-tracks", type=int, default=2, help="tracks timed alone on one thread")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the isolated STFT probe (A/B runs)")
    ap.add_argument("--bpm-mode", type=int, default=-1, help="synthetic BPM mix (-1 = the workload's; 1 = config 5)")
    ap.add_argument("--dry-run", action="store_true", help="host-logic rehearsal without a GPU (tests)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a box with fewer GPUs than ranks: every rank runs on device 0 (the "
                         "line is labelled; not a scaling measurement)")
    ap.add_argument("--rank-shard", type=int, default=-1,
                    help="config 3 on a one-GPU box: run rank R's shard of an 8-rank job (seeds R*tracks ..) "
                         "alone on device 0 (the line is labelled; not a scaling measurement)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    cfg_no, n_default, mix_default, stage_mask = WORKLOADS[args.workload]
    bpm_mode = mix_default if args.bpm_mode < 0 else args.bpm_mode
    eng = (DryEngine if args.dry_run else Engine)(0 if args.share_device else local)
    tdist = None
    if args.dry_run and os.environ.get("SDSP_BENCH_FAIL_RANK") == str(rank):
        raise SystemExit(3)  # test hook (dry runs only): this rank dies before the process group
    if world > 1:
        import torch.distributed as tdist

        tdist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if tdist is not None:
            tdist.barrier()

    sr = 44100
    n = args.tracks or n_default
    shard_rank = rank
    if args.rank_shard >= 0:
        if world != 1:
            raise SystemExit("bench.py: --rank-shard runs one shard in one process (--gpus 1)")
        shard_rank = args.rank_shard
    seed0 = shard_seed0(shard_rank, n)
    lens = track_lengths(args.workload, n, args.seconds, sr, seed0)
    buf, offs = eng.generate(lens, sr, seed0, bpm_mode)

    # results stay native (C-ABI structs, as a Rust/C caller receives them); the parity sample
    # below converts the tracks it checks
    for _ in range(args.warmup):
        eng.analyze(buf, offs, lens, sr, stage_mask).free()
    barrier()
    eng.synchronize()
    clock = ClockSampler(eng.dev) if (rank == 0 and not args.dry_run) else None
    if clock:
        clock.__enter__()
    t0 = time.perf_counter()
    stft = {"ms8": 0.0, "b8": 0.0, "l8": 0, "f8": 0, "ms2": 0.0, "b2": 0.0, "l2": 0, "f2": 0}
    step_s = []
    res = None
    for _ in range(args.steps):
        if res is not None:
            res.free()
        ts = time.perf_counter()
        res = eng.analyze(buf, offs, lens, sr, stage_mask)  # returns with the results on the host
        step_s.append(time.perf_counter() - ts)
        st = eng.stage_times()
        stft["ms8"] += st["stft8192_ms"]
        stft["b8"] += st["stft8192_bytes"]
        stft["l8"] += st["stft8192_launches"]
        stft["ms2"] += st["stft2048_ms"]
        stft["b2"] += st["stft2048_bytes"]
        stft["l2"] += st["stft2048_launches"]
        stft["f8"] += st.get("stft8192_frames", 0)
        stft["f2"] += st.get("stft2048_frames", 0)
    eng.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0, tdist)
    if clock:
        clock.__exit__(None, None, None)
    # every rank's shard (rank, tracks, first seed), gathered for the report: the ranks' tracks
    # must be disjoint and sum to the job's batch (config 3: 8 x 1024 = 8192)
    shard = {"rank": shard_rank, "tracks": n, "seed0": seed0}
    shards = [shard]
    if tdist is not None:
        shards = [None] * world
        tdist.all_gather_object(shards, shard)
    n_err = sum(1 for st in res.status if st != 0)
    total_tracks = n * world * args.steps
    value = total_tracks / dt
    stages = eng.stage_times()
    # roofline of the dominant STFT kernel: k_stft_slide8 (the 8192-point key STFT), or k_stft_slide<2048>
    # when the key path does not run (bpm-only).  Algorithmic bytes per launch (4*N_in +
    # 4*F*(nfft/2+1)) / average launch time (HIP events on the kernel's stream).
    key_k = stft["l8"] > 0
    tag = "8" if key_k else "2"
    nl = max(stft["l" + tag], 1)
    bytes_per_launch = stft["b" + tag] / nl
    ms_per_launch = stft["ms" + tag] / nl
    achieved = bytes_per_launch / (ms_per_launch * 1e-3) / 1e9 if ms_per_launch > 0 else 0.0
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_stft8192.json" if key_k else "pmc_stft2048.json")
    if os.path.exists(pmc_path):
        # rocprofv3 PMC passes (profiles/README.md): measured HBM bytes / algorithmic bytes for
        # this kernel; scales to the per-launch traffic of whatever batch this run used
        with open(pmc_path) as f:
            ratio = json.load(f).get("hbm_over_algorithmic")
        if ratio is not None:
            traffic = round(ratio * bytes_per_launch)
    roofline = {
        "bound": None,  # set below from the measured HBM and VALU-issue fractions
        "kernel": "k_stft_slide8w3 (key STFT, 8192/512)" if key_k else "k_stft_slide2s (tempo STFT, 2048/512)",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "bytes_per_launch": bytes_per_launch,
        "ms_per_launch": ms_per_launch,
        "launches": stft["l" + tag],
        "stft2048_GBps": round(stft["b2"] / (stft["ms2"] * 1e-3) / 1e9, 2) if stft["ms2"] > 0 else None,
        "stft_stage_GBps": round((stft["b2"] + stft["b8"]) / ((stft["ms2"] + stft["ms8"]) * 1e-3) / 1e9, 2)
        if (stft["ms2"] + stft["ms8"]) > 0 else None,
    }

    if not args.dry_run and rank == 0 and not args.no_probe:
        # the same kernel launched alone (nothing else on the chip): the kernel's own bandwidth, as
        # opposed to `achieved` above, which is measured inside the two-stream pipeline where the
        # tempo path shares the CUs (tools/stft_probe.py)
        roofline["isolated"] = isolated_stft(8192 if key_k else 2048, 512, int(lens.max()) if len(lens) else 0,
                                             sclk=clock.report() if clock else None)

    cpu = None
    parity = None
    extras = {}
    if clock and clock.report():
        extras["sclk_mhz_timed"] = clock.report()
    # The kernel's other roofline: VALU issue.  valu_frac = VALU wave-instructions the launches
    # issued (the frame loop's census from the kernel's ISA, profiles/isa_census_stft.json, x the
    # frames computed) / what the chip can issue in the launch time (1,024 SIMDs, one wave64 VALU
    # instruction per 2 cycles, MI355X_MICROARCH.md) at the 2,400 MHz peak clock (a lower bound;
    # the fraction at the sampled clock is reported beside it).  "bound" names the larger fraction.
    roofline.update(valu_roofline(key_k, stft, extras.get("sclk_mhz_timed")))
    roofline["bound"] = "valu-issue" if (roofline.get("valu_frac") or 0) > roofline["frac"] else "hbm"
    ss = sorted(step_s)
    extras["step_ms"] = {"median": round(1e3 * ss[len(ss) // 2], 3), "min": round(1e3 * ss[0], 3),
                         "max": round(1e3 * ss[-1], 3), "all": [round(1e3 * t, 3) for t in step_s]}
    if not args.dry_run:
        # fraction of this rank's tracks whose base estimate escalated to multi-resolution
        # (src/lib.rs:410-459; BASELINE.md asks for the escalation rate beside the throughput)
        extras["escalation_rate"] = round(res.count("tempogram_multi_res_triggered") / max(n, 1), 4)
        if stage_mask == 1:
            extras["bpm_only_vs_full"] = bpm_only_check(eng, buf, offs, lens, sr, res, min(n, 64))
    if args.workload == "mixed":
        extras["mean_track_seconds"] = round(float(lens.mean()) / sr, 2)
        extras["audio_seconds_per_s"] = round(float(lens.sum()) / sr * world * args.steps / dt, 1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run:
        cpu, parity = cpu_baseline(buf, offs, lens, res, n, sr, args)
        extras["sine_30s"] = sine_30s(sr)

    if rank == 0:
        wl = {
            "config2": f"batch of {n} synthetic {args.seconds:g}-s 44.1 kHz mono tracks per GPU, "
                       "AnalysisConfig::default(), full BPM + key + beat grid",
            "mixed": f"mixed-length batch of {n} synthetic tracks per GPU, whole seconds uniform in [30, 600] s, "
                     "AnalysisConfig::default(), full BPM + key + beat grid",
            "bpm-only": f"BPM-only path (stages a1-a19, multi-resolution escalation on) over {n} synthetic "
                        f"{args.seconds:g}-s tracks per GPU, BPMs 1/3 in [55,80], 1/3 in [170,200], 1/3 in [80,170]",
        }[args.workload]
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
            "data": "synthetic (seeded on-device generator: kick/hat/triad/diatonic line, 44.1 kHz mono)"
            + (" [DRY RUN: no GPU, not a measurement]" if args.dry_run else "")
            + (f" [REHEARSAL: {world} ranks sharing device 0, not a scaling measurement]" if args.share_device else "")
            + (f" [CONFIG-3 SHARD: rank {shard_rank}'s 1024-track seed range of the 8-GPU job, alone on device 0; "
               "not a scaling measurement]" if args.rank_shard >= 0 else ""),
            "config": {
                "workload": wl,
                "baseline_config": 3 if (cfg_no == 2 and (world > 1 or args.rank_shard >= 0)) else cfg_no,
                "tracks_per_gpu": n,
                "seconds_per_track": args.seconds if args.workload != "mixed" else "30-600",
                "sample_rate": sr,
                "bpm_mode": bpm_mode,
                "stages": "bpm-only (a1-a19)" if stage_mask == 1 else "full",
                "parallelism": f"track-sharded x{world} (no collectives)",
                "tracks_per_step_all_ranks": sum(x["tracks"] for x in shards),
                "shards": shards,
            },
            "errors": n_err,
            "stage_ms_last_step": {k: round(v, 3) for k, v in stages.items() if k.endswith("_ms")},
            # tracks of the last step analysed again with the sequential key-energy fold (their key
            # vote was near a decision under the block-folded energies)
            "key_reruns_last_step": int(stages.get("key_reruns", 0)),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity_sample": parity,
            **extras,
        }
        print(json.dumps(out), flush=True)
    if tdist is not None:
        tdist.destroy_process_group()


class ClockSampler:
    """Samples the shader clock of HIP device `dev` about once a second on a daemon thread while the
    timed steps run: the current level (the line marked *) of its card's sysfs pp_dpm_sclk, the
    card found by the device's PCI bus id (sdsp_debug_device_pci_bus_id), so HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES renumbering cannot point it at another card, and no subprocess runs inside
    the timed window.  The box runs bench processes in one of two clock states (~2.0 vs ~1.75 GHz,
    DESIGN.md §6), so the line reports which one it measured.  Absent the file, it reports nothing."""

    def __init__(self, dev=0):
        import threading

        self.mhz, self.stop, self.path = [], threading.Event(), None
        try:
            import ctypes as C

            b = C.create_string_buffer(64)
            L = sdsp.lib()
            L.sdsp_debug_device_pci_bus_id.argtypes = [C.c_int32, C.c_char_p, C.c_uint32]
            if L.sdsp_debug_device_pci_bus_id(dev, b, 64) == 0:
                p = os.path.join("/sys/bus/pci/devices", b.value.decode().lower(), "pp_dpm_sclk")
                if os.path.exists(p):
                    self.path, self.bus = p, b.value.decode().lower()
        except Exception:
            self.path = None
        self.th = threading.Thread(target=self._run, daemon=True) if self.path else None

    def _run(self):
        pat = re.compile(r"(\d+)\s*Mhz\s*\*", re.I)
        while not self.stop.is_set():
            try:
                with open(self.path) as f:
                    m = pat.search(f.read())
                if m:
                    self.mhz.append(int(m.group(1)))
            except OSError:
                return
            self.stop.wait(1.0)

    def __enter__(self):
        if self.th:
            self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        if self.th:
            self.th.join(timeout=15)

    def report(self):
        if not self.mhz:
            return None
        v = sorted(self.mhz)
        return {"median": v[len(v) // 2], "min": v[0], "max": v[-1], "samples": len(v),
                "source": f"sysfs pp_dpm_sclk of PCI {self.bus} (the HIP device's card)"}


CENSUS_KERNELS = {True: "k_stft_slide8w3ILi1E", False: "k_stft_slide2sILi4ELb1E"}


def valu_roofline(key_k, stft, sclk):
    """VALU-issue fraction of the dominant STFT kernel's launches (see the caller)."""
    path = os.path.join(ROOT, "profiles", "isa_census_stft.json")
    tag = "8" if key_k else "2"
    frames, ms, nl = stft["f" + tag], stft["ms" + tag], max(stft["l" + tag], 1)
    if not os.path.exists(path) or frames <= 0 or ms <= 0:
        return {"valu_frac": None}
    with open(path) as f:
        census = json.load(f)["kernels"]
    ent = next((v for k, v in census.items() if CENSUS_KERNELS[key_k] in k), None)
    if ent is None:
        return {"valu_frac": None}
    issued = ent["valu_per_frame"] * frames / nl

    def frac_at(mhz):
        return round(issued / ((ms / nl) * 1e-3 * 1024 * mhz * 1e6 / 2.0), 4)

    # the peak clock gives a lower bound of the issue fraction; the sysfs DPM level sampled during
    # the timed steps is reported beside it (MI355X_MICROARCH.md: the in-kernel clock can read up to
    # ~10 % below pp_dpm_sclk, and the probe runs after the sampled window)
    return {"valu_frac": frac_at(2400.0), "valu_frac_at_sampled_sclk": frac_at(float(sclk["median"])) if sclk else None,
            "valu_per_frame": ent["valu_per_frame"], "frames_per_launch": round(frames / nl, 1),
            "valu_method": "frame-loop VALU census from the kernel's ISA (tools/isa_census.py, "
                           "profiles/isa_census_stft.json) x frames / (launch time x 1024 SIMDs x 2,400 MHz / 2)"}


def isolated_stft(nfft, hop, length, tracks=256, reps=3, sclk=None):
    """sdsp_probe_stft: `reps` launches of the STFT kernel alone over `tracks` device-resident
    noise tracks of `length` samples, HIP events on its stream.  256 3-min tracks are 62k
    workgroups of the 8192-point kernel (80 per workgroup slot of the chip), so the launch measures
    the kernel and not its grid's tail; fewer when the device's free memory cannot hold them."""
    import ctypes as C

    if length < nfft:
        return None
    L = sdsp.lib()
    free = sdsp.device_mem_info(0)[0]
    frames = (length - nfft) // hop + 1
    per_track = 4 * length + 4 * frames * (4160 if nfft == 8192 else 1028) + 4 * frames
    tracks = int(max(8, min(tracks, 0.8 * free // per_track)))
    f = L.sdsp_probe_stft
    f.argtypes = [C.c_int32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32, C.c_int32,
                  C.POINTER(C.c_double), C.POINTER(C.c_double)]
    f.restype = C.c_int32
    ms, by = C.c_double(), C.c_double()
    stride = 4160 if nfft == 8192 else 1028  # the pipeline's row strides (pipeline.hip STRIDE8 / STRIDE2)
    if f(0, nfft, hop, tracks, length, reps, stride, C.byref(ms), C.byref(by)) != 0:
        return None
    gbs = by.value / (ms.value * 1e-3) / 1e9
    vr = valu_roofline(nfft == 8192, {"f8": tracks * frames, "ms8": ms.value, "l8": 1, "f2": tracks * frames,
                                      "ms2": ms.value, "l2": 1}, sclk)
    return {"kernel": "k_stft_slide8w3" if nfft == 8192 else "k_stft_slide2s", "tracks": tracks, "ms_per_launch": round(ms.value, 3),
            "valu_frac": vr.get("valu_frac"), "valu_frac_at_sampled_sclk": vr.get("valu_frac_at_sampled_sclk"),
            "ms_per_track": round(ms.value / tracks, 5), "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "method": "sdsp_probe_stft: the kernel launched alone on device-resident noise tracks of the workload's "
                      "length, HIP events, mean of 3 launches"}


def bpm_only_check(eng, buf, offs, lens, sr, res, k):
    """BASELINE config 5: the BPM-only stages must give a full run's bpm, bpm_confidence and
    multi-resolution flags.  Runs the full pipeline on the first k tracks and compares bitwise."""
    full = eng.analyze(buf, offs[:k], lens[:k], sr, 0)
    same = 0
    for i in range(k):
        a, b = res[i], full[i]
        if isinstance(a, Exception) or isinstance(b, Exception):
            same += int(type(a) is type(b))
            continue
        keys = ("bpm", "bpm_confidence")
        flags = ("tempogram_multi_res_triggered", "tempogram_multi_res_used")
        ok = all(np.float32(a[x]).tobytes() == np.float32(b[x]).tobytes() for x in keys)
        ok = ok and all(a["metadata"].get(f) == b["metadata"].get(f) for f in flags)
        same += int(ok)
    full.free()
    return {"checked": k, "identical": same}


def host_cpu():
    """The host the CPU baseline ran on: logical CPUs, the ones this process may use, the model."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    # the CPU share the job is granted: a GPU box hands each GPU a slice of the host and says so in
    # OMP_NUM_THREADS (its affinity set can still list every core of the machine)
    share = usable or 1
    try:
        share = min(share, int(os.environ.get("OMP_NUM_THREADS", "") or share))
    except ValueError:
        pass
    return {"nproc": os.cpu_count(), "usable": usable, "share": share, "model": model}


def cpu_baseline(buf, offs, lens, res, n, sr, args):
    """The oracle (C++ restatement, single-threaded per track, one track per thread as
    examples/analyze_batch.rs:239-268 does with rayon) on a bounded sample of the same tracks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import parity

    host = host_cpu()
    threads = args.cpu_threads or host["share"]
    k = min(n, args.cpu_tracks or threads)  # one track per thread
    xs = [buf.to_host(int(offs[i]), int(lens[i])) for i in range(k)]
    oracle.lib()

    def one(x):
        t = time.perf_counter()
        r = oracle.analyze(x, sr)  # ctypes releases the GIL: the threads run in parallel
        return r, time.perf_counter() - t

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(one, xs))
    dt = time.perf_counter() - t0
    per_track = [o[1] for o in outs]
    outs = [o[0] for o in outs]
    match = sum(1 for i, (st, ref) in enumerate(outs) if st == 0 and not parity.diff_results(res[i], ref))
    # bit_exact: every field bit for bit (strict); bit_exact_except_key_energy: every field but the
    # default key path's two block-folded energy fields, which diff_results checks
    # within the north star's 1e-4 (within_tolerance)
    exact = sum(1 for i, (st, ref) in enumerate(outs) if st == 0 and parity.exact_fraction(res[i], ref, strict=True) == 1.0)
    exact_nk = sum(1 for i, (st, ref) in enumerate(outs) if st == 0 and parity.exact_fraction(res[i], ref) == 1.0)
    key_eq = sum(1 for i, (st, ref) in enumerate(outs) if st == 0 and res[i]["key"] == ref["key"])
    cpu = {
        "value": round(k / dt, 4),
        "unit": "tracks/s",
        "cores": threads,
        "kind": "port",
        "host": host,
        "sample": f"{k} of the benchmark's own tracks, one track per thread on {threads} threads, "
                  f"{dt:.1f} s wall ({sum(per_track):.0f} thread-s); C++ restatement -O3, FFT per sdsp_fft_spec.h "
                  "(scalar radix-4; rustfft is SIMD)",
        # one thread's rate over the same k tracks, each timed inside its own thread (while the
        # other threads ran): k / the summed per-track seconds
        "value_1thread_loaded": round(k / sum(per_track), 4),
    }
    # the whole host, if every core ran one track at the loaded one-thread rate (an extrapolation,
    # stated as such: the job may use only its share of the host's cores)
    cpu["value_all_host_cores_extrapolated"] = round(cpu["value_1thread_loaded"] * (host["nproc"] or 1), 2)
    # one thread alone, the first tracks again (more than the parallel sample: its own tracks)
    k1 = max(1, args.cpu_1thread_tracks)
    if k1 > k:
        xs = xs + [buf.to_host(int(offs[i]), int(lens[i])) for i in range(k, min(n, k1))]
    k1 = min(k1, len(xs))
    t0 = time.perf_counter()
    for x in xs[:k1]:
        one(x)
    cpu["value_1thread"] = round(k1 / (time.perf_counter() - t0), 4)
    cpu["value_1thread_sample"] = f"{k1} tracks, alone on one thread"
    par = {"checked": k, "within_tolerance": match, "key_equal": key_eq, "bit_exact": exact,
           "bit_exact_except_key_energy": exact_nk}
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
