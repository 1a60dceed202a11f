#!/usr/bin/env python3
"""Isolated STFT kernel timing (sdsp_probe_stft) for one or more library builds.

    python tools/stft_probe.py [lib.so ...]      (default: the product library)

Prints, per library and STFT kind, ms per launch, ms per 3-min track and the HBM-roofline
fraction of the algorithmic bytes (4 N_in + 4 F (nfft/2+1)) against 8 TB/s.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "stratum-dsp_amd", "lib", "libstratum_hip.so")


def probe(path, nfft, hop, tracks, seconds=180.0, reps=3, stride=0):
    L = C.CDLL(path)
    f = L.sdsp_probe_stft
    f.argtypes = [C.c_int32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32, C.c_int32,
                  C.POINTER(C.c_double), C.POINTER(C.c_double)]
    f.restype = C.c_int32
    ms, by = C.c_double(), C.c_double()
    rc = f(0, nfft, hop, tracks, int(seconds * 44100), reps, stride, C.byref(ms), C.byref(by))
    if rc != 0:
        raise RuntimeError(f"sdsp_probe_stft rc={rc}")
    gbs = by.value / (ms.value * 1e-3) / 1e9
    return {"lib": os.path.basename(path), "nfft": nfft, "hop": hop, "tracks": tracks, "ms_per_launch": round(ms.value, 3),
            "ms_per_track": round(ms.value / tracks, 5), "GBps": round(gbs, 1), "frac": round(gbs / 8000.0, 4)}


if __name__ == "__main__":
    # SDSP_PROBE_TRACKS: tracks per launch (default 320 for 8192, 1024 for 2048: both fill the chip
    # many times over); SDSP_PROBE_ROUNDS: alternate the libraries this many times
    libs = sys.argv[1:] or [LIB]
    n8 = int(os.environ.get("SDSP_PROBE_TRACKS", "320"))
    rounds = int(os.environ.get("SDSP_PROBE_ROUNDS", "1"))
    only = os.environ.get("SDSP_PROBE_SIZES", "8192,2048").split(",")
    for _ in range(rounds):
        for lib in libs:
            for nfft, hop, n in ((8192, 512, n8), (2048, 512, 4 * n8)):
                if str(nfft) in only:
                    print(json.dumps(probe(lib, nfft, hop, n)), flush=True)
