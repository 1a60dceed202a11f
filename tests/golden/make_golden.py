#!/usr/bin/env python3
"""Regenerate tests/golden/oracle_results.json: the CPU restatement's AnalysisResult (serde
field names) on the reference's WAV fixtures and on 16 seeded synthetic tracks, plus per-stage
checksums of each (stages()).  These are the
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
SYNTH = [(0, 30.0), (1, 30.0), (2, 45.0), (3, 20.0)] + [(s, (20.0, 30.0, 45.0)[s % 3]) for s in range(4, 16)]


def stages(x, sr):
    """Per-stage checksums of the oracle on one track: trim (a3), the onset
    lists (a4, a6-a8), the full novelty curve (a10-a13, from the trimmed track's 2048/512 STFT),
    the base tempogram estimate and its top-5 candidates (a14-a16), the escalation flags (a17-a18),
    the beat-grid branches (a20-a23) and the key-stage arrays (a24-a27)."""
    import numpy as np

    st, r, tr = oracle.analyze(x, sr, trace=True)
    assert st == 0
    _, xn = oracle.normalize(x, 0, sr)
    nov = oracle.novelty_full(oracle.stft(xn[tr["trim_start"]:tr["trim_end"]], 2048, 512), sr).astype(np.float64)
    out = {"trim": [tr["trim_start"], tr["trim_end"]]}
    for k in ("energy_onsets", "spectral_onsets", "hfc_onsets", "chosen_onsets"):
        out[k] = [len(tr[k]), int(sum(tr[k]))]
    out["novelty"] = [int(nov.size), float(nov.sum()), float((nov * nov).sum()), int(nov.argmax()) if nov.size else -1]
    out["base"] = tr["base"]
    out["base_top5"] = tr["base_cands"][:5]
    out["escalation"] = [tr["ambiguous"], tr["ran_mr"], tr["used_mr"], tr["mr"]]
    out["beat"] = [tr["beat_variable"], tr["beat_refined"], tr["beats_per_bar"]]
    out["key"] = [tr["n_key_frames"], tr["chroma_sum"], tr["chroma_sq"], tr["energy_sum"], tr["weights_sum"],
                  tr["weights_used"], tr["used_segments"]]
    return out


def strip(r):
    r = dict(r)
    r["metadata"] = {k: v for k, v in r["metadata"].items() if k != "processing_time_ms"}
    return r


def main():
    out = {"fixtures": {}, "synthetic": {}, "stages": {}}
    for name in FIXTURES:
        x, sr = parity.load_wav(os.path.join(HERE, name))
        st, r = oracle.analyze(x, sr)
        assert st == 0, (name, r)
        out["fixtures"][name] = strip(r)
        out["stages"][name] = stages(x, sr)
    for seed, sec in SYNTH:
        x, *_ = synth.make_track(seed, seconds=sec)
        st, r = oracle.analyze(x, 44100)
        assert st == 0
        out["synthetic"][f"{seed}:{sec:g}"] = strip(r)
        out["stages"][f"{seed}:{sec:g}"] = stages(x, 44100)
    with open(os.path.join(HERE, "oracle_results.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
