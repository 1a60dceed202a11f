#!/usr/bin/env python3
"""Where the default key path's block-folded HPCP energies change a key decision:
the oracle run twice on one track, with the reference's sequential frame-energy fold and with the
GPU's 64-bin block fold (the oracle's study switch), and the key vote's per-segment raw scores and
clarities compared.

    python tools/key_near_study.py TRACK.npy [TRACK.npy ...]

Per track: the results' key / key_confidence / key_clarity under both folds; per segment the largest
relative change of a raw score, the change of the clarity, the clarity's distance to the 0.2 gate,
the within-mode top-two relative gaps, and every segment whose gate decision or within-mode argmax
differs between the folds.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stratum-dsp_amd", "python"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402


def run(x, block):
    L = oracle.lib()
    L.sdsp_oracle_study_block_energy(int(block))
    L.sdsp_oracle_study_key_trace(1)
    st, r = oracle.analyze(x, 44100)
    L.sdsp_oracle_study_key_trace_get.restype = C.c_uint64
    n = L.sdsp_oracle_study_key_trace_get(None, 0)
    buf = np.zeros(n, np.float32)
    L.sdsp_oracle_study_key_trace_get(buf.ctypes.data_as(C.POINTER(C.c_float)), C.c_uint64(n))
    L.sdsp_oracle_study_key_trace(0)
    L.sdsp_oracle_study_block_energy(0)
    return r, buf


def segments(tr):
    """(raw[24], clarity) per segment of segment voting: records of 25 floats."""
    k = len(tr) // 25
    return [(tr[25 * i:25 * i + 24], float(tr[25 * i + 24])) for i in range(k)]


def gaps(raw):
    out = []
    for m in range(2):
        v = np.sort(raw[12 * m:12 * m + 12])[::-1]
        out.append(float((v[0] - v[1]) / v[0]) if v[0] > 0 else 0.0)
    return out


def main():
    for path in sys.argv[1:]:
        x = np.load(path).astype(np.float32)
        re, te = run(x, False)
        rb, tb = run(x, True)
        se, sb = segments(te), segments(tb)
        rep = {"track": os.path.basename(path), "exact": [re["key"], re["key_confidence"], re["key_clarity"]],
               "block": [rb["key"], rb["key_confidence"], rb["key_clarity"]], "segments": len(se),
               "max_rel_score_change": 0.0, "max_clarity_change": 0.0, "min_gate_distance": 1.0,
               "min_within_mode_gap": 1.0, "gate_flips": [], "argmax_flips": []}
        for i, ((ra, ca), (rb_, cb)) in enumerate(zip(se, sb)):
            rel = np.max(np.abs(ra - rb_) / np.maximum(np.abs(ra), 1e-30))
            rep["max_rel_score_change"] = max(rep["max_rel_score_change"], float(rel))
            rep["max_clarity_change"] = max(rep["max_clarity_change"], abs(ca - cb))
            rep["min_gate_distance"] = min(rep["min_gate_distance"], abs(ca - 0.2))
            rep["min_within_mode_gap"] = min(rep["min_within_mode_gap"], *gaps(ra))
            if (ca >= 0.2) != (cb >= 0.2):
                rep["gate_flips"].append([i, ca, cb])
            for m in range(2):
                if int(np.argmax(ra[12 * m:12 * m + 12][::-1])) != int(np.argmax(rb_[12 * m:12 * m + 12][::-1])):
                    rep["argmax_flips"].append([i, m, gaps(ra)[m]])
        print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
