"""Per-phase clock of k_key_vote (the SDSP_KV_PROF build prints one line per 64th workgroup) on a
batch of n 3-min tracks from the bench generator: python3 tools/kv_prof.py <n>"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stratum-dsp_amd", "python")]
import numpy as np
import sdsp
n = int(sys.argv[1]); L = 180 * 44100
buf = sdsp.DeviceBuffer(n * L)
sdsp.generate_synthetic(buf.ptr, n, L, 44100, seed0=0)
for rep in range(2):
    sdsp.analyze_batch_device(buf.ptr, np.arange(n) * L, np.full(n, L), 44100)
    print("stage", {k: v for k, v in sdsp.stage_times().items() if "rerun" in k or "key" in k}, flush=True)
