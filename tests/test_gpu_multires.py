"""Multi-resolution escalation off the default hop and without the auxiliary tempogram variants
(GPU, through the C ABI), against the oracle.

The reference's escalation (src/lib.rs:489-575 -> multi_resolution.rs:205-901) recomputes the
STFT at hops 256, 512 and 1024 of the trimmed samples whatever hop_size is (:237-239), takes the
hop-512 list with top_k candidates (:273) and gates its folds with the hop-512 novelty made with
the configured weights (:680-694), which differ from combined_novelty's defaults the base
tempogram uses when band fusion, mel novelty and the consensus bonus are all off.  The engine runs
its own hop-512 pass for the escalated tracks when hop_size != 512 and a second hop-512 novelty
when the variants are off; the oracle follows the reference directly.  Tracks are an
escalation-heavy BPM mix (slow, fast and mid tempos) and the test asserts escalation happened.
"""
import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu

NO_AUX = dict(enable_tempogram_band_fusion=0, enable_tempogram_mel_novelty=0, tempogram_band_consensus_bonus=0.0)
CASES = {
    "hop256": dict(hop_size=256),
    "hop1024": dict(hop_size=1024),
    "hop441": dict(hop_size=441),  # not a sliding-STFT hop: the frame-parallel STFT path
    "hop1024_candidates": dict(hop_size=1024, emit_tempogram_candidates=1),
    "no_aux_hop512": dict(NO_AUX),
    "no_aux_hop1024": dict(NO_AUX, hop_size=1024),
    "no_aux_candidates": dict(NO_AUX, emit_tempogram_candidates=1),
}
BPMS = [62.0, 68.0, 74.0, 176.0, 184.0, 195.0, 92.0, 128.0]

_TRACKS = None


def tracks():
    global _TRACKS
    if _TRACKS is None:
        _TRACKS = [synth.make_track(500 + k, seconds=45.0, bpm=b)[0] for k, b in enumerate(BPMS)]
    return _TRACKS


def _cfg(base, opts):
    for k, v in opts.items():
        setattr(base, k, v)
    return base


@pytest.mark.parametrize("case", sorted(CASES))
def test_multires_config_parity(case):
    cfg = _cfg(sdsp.default_config(), CASES[case])
    ocfg = _cfg(oracle.default_config(), CASES[case])
    xs = tracks()
    got = sdsp.analyze_batch(xs, 44100, cfg)
    trig = 0
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, ocfg)
        assert st == 0, (case, i, ref)
        assert not isinstance(got[i], Exception), (case, i, got[i])
        bad = parity.diff_results(got[i], ref)
        assert not bad, f"{case} track {i}: {bad}"
        assert parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, (case, i)
        trig += ref["metadata"].get("tempogram_multi_res_triggered") is True
    assert trig >= 2, (case, trig)  # the escalation path is exercised


def test_multires_hop_changes_results():
    """hop_size is live on the escalation path: some bpm / confidence / flag differs from hop 512."""
    xs = tracks()
    a = sdsp.analyze_batch(xs, 44100, sdsp.default_config())
    b = sdsp.analyze_batch(xs, 44100, _cfg(sdsp.default_config(), dict(hop_size=1024)))
    diff = sum(1 for r, s in zip(a, b) if (r["bpm"], r["bpm_confidence"]) != (s["bpm"], s["bpm_confidence"]))
    assert diff >= 1
    assert all(np.isfinite(r["bpm"]) for r in b)
