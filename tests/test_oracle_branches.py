"""Branch coverage of the CPU restatement on inputs that reach the reference's rarely taken
paths, with the branch read from the oracle's trace / result flags.  CPU only; the GPU tests run
the same inputs and compare every field bit-exactly (tests/test_gpu_hpss.py, test_gpu_parity.py).

- percussive tempogram fallback accepted (src/lib.rs:587-683): synth.chord_stab_track with
  enable_tempogram_percussive_fallback; the same track without the fallback keeps the base BPM
- tempo variation -> Bayesian refinement (beat_tracking/mod.rs:152-219): seeded synthetic tracks
  whose HMM beats have a variable segment (also cross-checked by tests/test_ref64.py)
"""
import numpy as np

import oracle
import synth


def test_percussive_fallback_accepted():
    x = synth.chord_stab_track()
    cfg = oracle.default_config()
    cfg.enable_tempogram_percussive_fallback = 1
    st, r, tr = oracle.analyze(x, 44100, config=cfg, trace=True)
    assert st == 0
    md = r["metadata"]
    assert md["tempogram_multi_res_triggered"] is True and md["tempogram_percussive_triggered"] is True
    assert md["tempogram_percussive_used"] is True
    assert 55.0 <= tr["base"][0] <= 80.0  # base estimate in the low trap zone
    assert abs(r["bpm"] / tr["base"][0] - 2.0) < 0.05  # the accepted estimate is the double-time family
    st, r0 = oracle.analyze(x, 44100)
    assert st == 0 and r0["metadata"]["tempogram_percussive_used"] is None  # fallback off: flags stay None


def test_bayesian_refinement_taken():
    taken = 0
    for seed in range(4):
        x, *_ = synth.make_track(seed, seconds=30.0)
        st, r, tr = oracle.analyze(x.astype(np.float32), 44100, trace=True)
        assert st == 0
        taken += bool(tr["beat_variable"]) and bool(tr["beat_refined"])
    assert taken >= 1
