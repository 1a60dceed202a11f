#!/usr/bin/env python3
"""Regenerate tests/golden/oracle_results.json: the CPU restatement's AnalysisResult (serde
field names) on the reference's WAV fixtures and on seeded synthetic tracks.  These are the
golden vectors the GPU engine is checked against (tests/test_gpu_parity.py) and that pin the
oracle itself between rounds (tests/test_oracle_integration.py).  Run from the repo root:
    python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "stratum-dsp_amd", "python")]

import oracle  # noqa: E402
import parity  # noqa: E402
import synth  # noqa: E402

FIXTURES = ["120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"]
SYNTH = [(0, 30.0), (1, 30.0), (2, 45.0), (3, 20.0)]


def strip(r):
    r = dict(r)
    r["metadata"] = {k: v for k, v in r["metadata"].items() if k != "processing_time_ms"}
    return r


def main():
    out = {"fixtures": {}, "synthetic": {}}
    for name in FIXTURES:
        x, sr = parity.load_wav(os.path.join(HERE, name))
        st, r = oracle.analyze(x, sr)
        assert st == 0, (name, r)
        out["fixtures"][name] = strip(r)
    for seed, sec in SYNTH:
        x, *_ = synth.make_track(seed, seconds=sec)
        st, r = oracle.analyze(x, 44100)
        assert st == 0
        out["synthetic"][f"{seed}:{sec:g}"] = strip(r)
    with open(os.path.join(HERE, "oracle_results.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
