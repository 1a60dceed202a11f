"""The default key path's block-folded energies (k_mask_rp / k_hpcp_band) against the oracle on
synthetic tracks and the reference fixtures: every field but key_confidence / key_clarity
bit-exact, the key equal, those two within 1e-4; prints how many tracks are bit-exact overall.
usage: python tools/key_band_check.py [n_tracks]"""
import os
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stratum-dsp_amd", "python"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import parity  # noqa: E402
import sdsp  # noqa: E402
import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
xs = [synth.make_track(7000 + k, seconds=30.0 + 5 * (k % 7))[0] for k in range(n)]
for f in ("120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"):
    xs.append(parity.load_wav(os.path.join(ROOT, "tests", "golden", f))[0])
res = sdsp.analyze_batch(xs, strict=False)
out = {"tracks": len(xs), "key_equal": 0, "within_tol": 0, "bit_exact_all": 0, "bit_exact_nonkey": 0,
       "max_key_conf_diff": 0.0, "max_key_clarity_diff": 0.0, "bad": []}
for i, (x, r) in enumerate(zip(xs, res)):
    st, ref = oracle.analyze(x, 44100)
    if st != 0 or isinstance(r, Exception):
        out["bad"].append([i, "error", str(r)])
        continue
    out["key_equal"] += int(r["key"] == ref["key"])
    d = parity.diff_results(r, ref)
    out["within_tol"] += int(not d)
    if d:
        out["bad"].append([i, d])
    out["bit_exact_all"] += int(parity.exact_fraction(r, ref) == 1.0)
    g, e = parity.result_digest(r), parity.result_digest(ref)
    out["bit_exact_nonkey"] += int(all(g[k] == e[k] for k in g if k not in ("key_confidence", "key_clarity")))
    out["max_key_conf_diff"] = max(out["max_key_conf_diff"], abs(r["key_confidence"] - ref["key_confidence"]))
    out["max_key_clarity_diff"] = max(out["max_key_clarity_diff"], abs(r["key_clarity"] - ref["key_clarity"]))
print(json.dumps(out))
