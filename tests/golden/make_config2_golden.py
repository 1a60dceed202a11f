"""Writes tests/golden/config2_oracle.json: the CPU restatement's results (bit-level digests,
parity.result_digest) on 64 device-generated 3-min 44.1 kHz tracks (sdsp_generate_synthetic,
seeds 3000..3063, BASELINE config 2's track shape), with a SHA-256 of each track's samples so the
test can prove it analyses the same input.  The generator runs on the GPU, so this script runs
on the MI355X box (from the repo root):

    python3 tests/golden/make_config2_golden.py [out.json]

The oracle (oracle/build/libsdsp_oracle.so) is the checker; the HIP engine only generates the
samples here.  tests/test_gpu_batch_paths.py::test_config2_shaped_sub_batches reads the file.
"""
import concurrent.futures as cf
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("oracle", "tests", os.path.join("stratum-dsp_amd", "python")):
    sys.path.insert(0, os.path.join(ROOT, p))

import oracle  # noqa: E402
import parity  # noqa: E402
import sdsp  # noqa: E402

N, L, SEED0 = 64, 44100 * 180, 3000


def main():
    buf = sdsp.DeviceBuffer(N * L)
    sdsp.generate_synthetic(buf.ptr, N, L, seed0=SEED0)
    xs = [buf.to_host(i * L, L) for i in range(N)]
    oracle.lib()
    with cf.ThreadPoolExecutor(16) as ex:
        outs = list(ex.map(lambda x: oracle.analyze(x, 44100), xs))
    tracks = []
    for x, (st, ref) in zip(xs, outs):
        assert st == 0, ref
        tracks.append({"samples": parity.samples_digest(x), "result": parity.result_digest(ref)})
    out = {"n": N, "length": L, "seed0": SEED0, "generator": "sdsp_generate_synthetic bpm_mode 0",
           "checker": "oracle (C++ restatement)", "tracks": tracks}
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "config2_oracle.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path)


if __name__ == "__main__":
    main()
