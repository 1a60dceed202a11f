"""The chunk queue behind sdsp_analyze_batch (stratum-dsp_amd/csrc/batch_sched.hpp) with fake
devices, on the CPU.  It replaces the reference's caller-side per-track fan-out
(examples/analyze_batch.rs:239-268) and shards chunks over GPUs with no collective.
The same header is compiled into libstratum_hip.so; here a host harness (tests/cpp/
batch_sched_test.cpp) checks that every track is analysed exactly once and lands in its own
output slot, that failed chunks are reported per chunk, and that a device whose copier dies
hands its work to the others."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = tmp_path_factory.mktemp("bsched") / "batch_sched_test"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-pthread", "-Wall", "-o", str(exe),
                           os.path.join(ROOT, "tests", "cpp", "batch_sched_test.cpp")])
    return str(exe)


@pytest.mark.parametrize("scenario", ["basic", "single", "analyze_fails", "copier_dies", "all_copiers_die",
                                      "copier_throws_int", "analyze_throws_int"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_chunk_queue(harness, scenario, seed):
    out = subprocess.run([harness, scenario, str(seed)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, (out.returncode, out.stdout, out.stderr)
    assert out.stdout.startswith("ok " + scenario)
    if scenario in ("basic", "analyze_fails"):
        assert "devices_used=3" in out.stdout  # work spread over every fake device
