"""Throughput of the GPU path under opt-in configurations, beside the default.

    python tools/config_cost.py [--tracks 1024] [--seconds 180] [--steps 3] [case ...]

Each case is a set of AnalysisConfig overrides; the same resident batch of synthetic tracks
(the bench generator) is analysed `steps` times per case after one warmup, and the tracks/s and
the per-stage times of the last call are printed as one JSON line per case.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stratum-dsp_amd", "python"))
import sdsp  # noqa: E402

_KEEP = []
CASES = {
    "default": {},
    "rms": dict(normalization=1),
    "lufs": dict(normalization=2),
    "key_sharpen_trim_temperley": dict(chroma_sharpening_power=2.0, enable_key_edge_trim=1, key_template_set=1),
    "key_ensemble": dict(enable_key_ensemble=1),
    "key_mode_heuristic": dict(enable_key_mode_heuristic=1, enable_key_minor_harmonic_bonus=1),
    "key_multi_scale": dict(enable_key_multi_scale=1),
    "hpss_onsets": dict(enable_hpss_onsets=1),
    "percussive_fallback": dict(enable_tempogram_percussive_fallback=1),
    "force_legacy": dict(force_legacy_bpm=1),
    "bpm_fusion": dict(enable_bpm_fusion=1),
    "key_hpss": dict(enable_key_hpss_harmonic=1),
}


def apply(cfg, opts):
    for k, v in opts.items():
        if isinstance(v, list):
            arr = np.ascontiguousarray(v, dtype=np.uint64 if k.endswith("lengths") else np.float32)
            _KEEP.append(arr)
            setattr(cfg, k, arr.ctypes.data_as(C.POINTER(C.c_uint64 if k.endswith("lengths") else C.c_float)))
            setattr(cfg, k + "_len", arr.size)
        else:
            setattr(cfg, k, v)
    return cfg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=1024)
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("cases", nargs="*")
    a = ap.parse_args()
    sr, n = 44100, a.tracks
    L = int(a.seconds * sr)
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, sr, seed0=1)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, dtype=np.uint64)
    for name in a.cases or list(CASES):
        cfg = apply(sdsp.default_config(), CASES[name])
        sdsp.analyze_batch_device(buf.ptr, offs, lens, sr, config=cfg, raw=True).free()
        sdsp.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            sdsp.analyze_batch_device(buf.ptr, offs, lens, sr, config=cfg, raw=True).free()
        sdsp.synchronize()
        dt = time.perf_counter() - t0
        st = sdsp.stage_times(0)
        print(json.dumps({"case": name, "tracks_per_s": round(n * a.steps / dt, 1),
                          "ms_per_step": round(dt / a.steps * 1e3, 2),
                          "stage_ms": {k: round(v, 2) for k, v in st.items() if k.endswith("_ms")}}), flush=True)


if __name__ == "__main__":
    main()
