"""PCIe-inclusive rate of the host-buffer API (sdsp_analyze_batch): N synthetic 3-min tracks are
generated on the device, copied to host memory, then analysed from host buffers (timed, 2 runs
after a warmup).  Prints one JSON line.  Usage: python tools/host_batch_rate.py [N]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stratum-dsp_amd", "python"))
import sdsp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
L = 44100 * 180
buf = sdsp.DeviceBuffer(n * L)
sdsp.generate_synthetic(buf.ptr, n, L, seed0=0)
host = buf.to_host()
del buf
tracks = [host[i * L:(i + 1) * L] for i in range(n)]
sdsp.analyze_batch(tracks[:64], 44100)
ts = []
for _ in range(2):
    t0 = time.perf_counter()
    res = sdsp.analyze_batch(tracks, 44100)
    ts.append(time.perf_counter() - t0)
ok = sum(1 for r in res if not isinstance(r, sdsp.AnalysisError))
print(json.dumps({"host_buffer_tracks_per_s": round(n / min(ts), 2), "tracks": n, "ok": ok,
                  "seconds": [round(t, 3) for t in ts]}))
