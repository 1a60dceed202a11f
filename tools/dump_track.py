#!/usr/bin/env python3
"""Save one device-generated synthetic track (the bench's generator) to gpurun_out/t<seed>_<mode>.npy,
so a GPU-box track can be studied on the CPU with the oracle.
usage: python tools/dump_track.py SEED BPM_MODE [SECONDS]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stratum-dsp_amd", "python")]
import sdsp  # noqa: E402

seed, mode = int(sys.argv[1]), int(sys.argv[2])
n = int(float(sys.argv[3] if len(sys.argv) > 3 else 180.0) * 44100)
# the generator's BPM mix of mode 1 takes the track's index in the call modulo 3: generate from the
# last multiple of 3 so the track is the one a batch starting at seed 0 holds (bench, key_scale_check)
k = seed % 3 + 1
buf = sdsp.DeviceBuffer(k * n)
sdsp.generate_synthetic(buf.ptr, k, n, 44100, seed0=seed - (k - 1), bpm_mode=mode)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"t{seed}_{mode}.npy"), buf.to_host((k - 1) * n, n))
print("ok", seed, mode, n)
