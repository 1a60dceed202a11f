"""The N>1 path on the CPU (gloo, world size 2, 127.0.0.1).  The path shards by track with no
data-path collective: each rank owns a disjoint contiguous seed range, the job
time is the slowest rank's, and rank 0 alone reports the whole-job throughput.
"""
import json
import os
import socket
import subprocess
import time
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch.distributed as tdist

    import bench

    tdist.init_process_group("gloo", rank=rank, world_size=world)
    seed0 = bench.shard_seed0(rank, 16)
    dt = bench.max_over_ranks(0.5 + rank, tdist)  # rank 1 is the slow one
    q.put((rank, seed0, dt))
    tdist.destroy_process_group()


def test_sharding_and_max_over_ranks():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert [g[1] for g in got] == [0, 16]          # disjoint contiguous track ranges
    assert all(abs(g[2] - 1.5) < 1e-12 for g in got)  # every rank sees the slowest time


def test_bench_launcher_world2_dry_run():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--tracks", "4", "--seconds", "1", "--dry-run"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 2 - 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    assert abs(d["value"] - 4 * 2 * 2 / (d["ms_per_step"] * 2 / 1000.0)) / d["value"] < 1e-2
    assert d["config"]["parallelism"].startswith("track-sharded x2")


def _bench_json(cmd):
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    return json.loads(lines[0])


def test_bench_spawns_ranks_without_torchrun():
    """`python bench.py --gpus 2` (the driver's plain invocation) starts its own 2 rank processes."""
    d = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                     "--tracks", "3", "--seconds", "1", "--dry-run"])
    assert d["n_gpus"] == 2 and d["steps"] == 2
    assert d["config"]["parallelism"].startswith("track-sharded x2")
    assert d["config"]["baseline_config"] == 3
    assert abs(d["value"] - 3 * 2 * 2 / (d["ms_per_step"] * 2 / 1000.0)) / d["value"] < 1e-2
    assert len(d["step_ms"]["all"]) == 2


def test_bench_spawned_rank_failure_ends_the_job():
    """A rank that dies before the barrier ends its siblings (which would otherwise wait in gloo)
    and the parent exits with its status instead of hanging."""
    env = dict(os.environ, SDSP_BENCH_FAIL_RANK="1")
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                          "--tracks", "2", "--seconds", "1", "--dry-run"], capture_output=True, text=True, timeout=200,
                         cwd=ROOT, env=env)
    assert out.returncode == 3, (out.returncode, out.stderr[-1000:])
    assert time.time() - t0 < 150


@pytest.mark.parametrize("workload,cfg", [("mixed", 4), ("bpm-only", 5)])
def test_bench_workloads_dry_run(workload, cfg):
    d = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--steps", "1",
                     "--warmup", "0", "--tracks", "5", "--dry-run"])
    assert d["n_gpus"] == 1 and d["config"]["baseline_config"] == cfg
    assert d["config"]["stages"] == ("bpm-only (a1-a19)" if workload == "bpm-only" else "full")


def test_mixed_lengths_are_config4():
    sys.path.insert(0, ROOT)
    import bench

    a = bench.track_lengths("mixed", 2000, 180.0, 44100, 0)
    assert a.min() >= 30 * 44100 and a.max() <= 600 * 44100 and (a % 44100 == 0).all()
    assert len(set((a // 44100).tolist())) > 400  # spread over the whole range
    b = bench.track_lengths("mixed", 2000, 180.0, 44100, 2000)
    assert not (a == b).all()  # ranks draw different tracks


def test_gpus_world_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--tracks", "2",
                          "--seconds", "1"], capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_bench_spawns_eight_ranks_without_torchrun():
    """The driver's 8-GPU invocation, rehearsed on the CPU: 8 rank processes, one JSON line, the
    whole job's tracks over the slowest rank's time."""
    d = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "0",
                     "--tracks", "2", "--seconds", "1", "--dry-run"])
    assert d["n_gpus"] == 8 and d["config"]["parallelism"].startswith("track-sharded x8")
    assert d["config"]["baseline_config"] == 3
    assert abs(d["value"] - 2 * 8 / (d["ms_per_step"] / 1000.0)) / d["value"] < 1e-2


def test_bench_eight_ranks_config3_shards():
    """Config 3 rehearsed on the CPU (BASELINE.json: 8192 tracks over 8 GPUs): the rank-0 line says
    n_gpus 8 and baseline config 3, and its per-rank shards are 8 disjoint seed ranges of 1024
    tracks, 8192 in all."""
    d = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "0",
                     "--seconds", "1", "--dry-run"])
    c = d["config"]
    assert d["n_gpus"] == 8 and c["baseline_config"] == 3 and c["tracks_per_gpu"] == 1024
    sh = sorted(c["shards"], key=lambda x: x["rank"])
    assert [x["rank"] for x in sh] == list(range(8)) and all(x["tracks"] == 1024 for x in sh)
    assert c["tracks_per_step_all_ranks"] == 8192 == sum(x["tracks"] for x in sh)
    ranges = sorted((x["seed0"], x["seed0"] + x["tracks"]) for x in sh)
    assert all(a[1] <= b[0] for a, b in zip(ranges, ranges[1:]))  # disjoint


def test_bench_share_device_rehearsal_is_labelled():
    """--share-device (a multi-rank rehearsal on a box with fewer GPUs than ranks: every rank on
    device 0) labels its line, so it cannot pass for a scaling measurement."""
    d = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                     "--tracks", "2", "--seconds", "1", "--dry-run", "--share-device"])
    assert d["n_gpus"] == 2 and "REHEARSAL: 2 ranks sharing device 0" in d["data"]


def test_bench_rank_shard_is_labelled_config3():
    """--rank-shard R (config 3 on a one-GPU box): one process runs rank R's seed range of the
    8-rank job on device 0; the line says baseline config 3, names the shard and is labelled as
    not a scaling measurement."""
    d = _bench_json([sys.executable, os.path.join(ROOT, "bench.py"), "--rank-shard", "5", "--steps", "1", "--warmup",
                     "0", "--tracks", "4", "--seconds", "1", "--dry-run"])
    c = d["config"]
    assert d["n_gpus"] == 1 and c["baseline_config"] == 3
    assert c["shards"] == [{"rank": 5, "tracks": 4, "seed0": 20}]
    assert "CONFIG-3 SHARD: rank 5" in d["data"]
