"""The default key path's block-folded frame energies (k_mask_rp + k_hpcp_band).

HPCP needs the masked 8192-point spectrogram only on its peak band, but folds every frame's energy
sum(x * x) over all 4,097 bins (extractor.rs:1133).  The engine's mask kernel stores the masked
values on the band only and folds each frame's squares in 64-bin blocks, HPCP folds the 65 block
sums: the one f32 sum is re-associated, every masked value and every other stage is unchanged.
The north star's tolerance (key exact, confidences within 1e-4) is what the key fields are held to;
every other field stays bit-identical to the oracle.  The config-2 golden (64 x 3-min) is checked
the same way in test_gpu_batch_paths.py.
"""
import concurrent.futures as cf

import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu


def _tracks():
    xs = [synth.make_track(9100 + k, seconds=20.0 + 7 * (k % 9), mode=k % 2, tonic=(5 * k) % 12)[0] for k in range(40)]
    xs += [synth.make_track(9200 + k, seconds=180.0)[0] for k in range(4)]
    return xs


def test_block_energies_key_exact_fields_bitexact():
    xs = _tracks()
    got = sdsp.analyze_batch(xs)
    n_key_bits = 0
    worst = 0.0
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100)
        assert st == 0, i
        assert got[i]["key"] == ref["key"], (i, got[i]["key"], ref["key"])
        assert not parity.diff_results(got[i], ref), (i, parity.diff_results(got[i], ref))
        g, e = parity.result_digest(got[i]), parity.result_digest(ref)
        assert all(g[k] == e[k] for k in g if k not in parity.KEY_ENERGY_FIELDS), i
        n_key_bits += int(all(g[k] == e[k] for k in parity.KEY_ENERGY_FIELDS))
        worst = max(worst, abs(got[i]["key_confidence"] - ref["key_confidence"]),
                    abs(got[i]["key_clarity"] - ref["key_clarity"]))
    print(f"key-energy fields bit-equal on {n_key_bits} of {len(xs)} tracks; worst |diff| {worst:.3g}")
    assert worst <= parity.TOL


def test_exact_energy_configs_stay_bitexact():
    """Configurations the band path does not serve keep k_mask_r + the full-spectrum HPCP walk,
    bit-identical to the oracle in every field (here: a mask margin other than 12)."""
    cfg = sdsp.default_config()
    cfg.key_spectrogram_smooth_margin = 8
    xs = [synth.make_track(9300 + k, seconds=25.0 + 4 * k)[0] for k in range(4)]
    got = sdsp.analyze_batch(xs, config=cfg)
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, config=cfg)
        assert st == 0 and parity.exact_fraction(got[i], ref, strict=True) == 1.0, i



def test_near_decision_track_rerun_exact():
    """Track 538 of BASELINE config 5's mix (bench.py's generator, bpm_mode 1; the mix picks the
    BPM range by the track's index in the call, so it is generated as the second of two tracks from
    seed 537).  Under the block-folded energies one segment's within-mode argmax flips (a top-two
    gap of 6.6e-7, tools/key_near_study.py) and key_confidence came out 0.0058 against the
    oracle's 0.0086 (profiles/r05_key_scale_block_energies.jsonl).  k_key_vote flags it
    (KeyOut::near) and the library analyses it again with the sequential fold: every field
    bit-exact, the rerun reported in the stage times and by sdsp_debug_last_key_near."""
    n = 180 * 44100
    buf = sdsp.DeviceBuffer(2 * n)
    sdsp.generate_synthetic(buf.ptr, 2, n, 44100, seed0=537, bpm_mode=1)
    got = sdsp.analyze_batch_device(buf.ptr, [n], [n], 44100)
    st = sdsp.stage_times()
    assert st["key_reruns"] == 1 and sdsp.last_key_near(1)[0] & 1  # the within-mode argmax margin
    rc, ref = oracle.analyze(buf.to_host(n, n), 44100)
    assert rc == 0
    assert parity.exact_fraction(got[0], ref, strict=True) == 1.0 and not parity.diff_results(got[0], ref)


def test_rigorous_certificate_covers_fixed_margins():
    """The rigorous certificate (per-frame energy bounds from k_hpcp_band carried
    through the weights, raw scores, clarities and the vote) flags every track the round-5 fixed
    margins flag (they are its floors), and on this batch of 3-min tracks from the bench's generator
    every result equals the oracle: key exact, every other field bit-exact, the two energy-weighted
    fields within the tolerance (flagged tracks bit-exact: they were rerun with the sequential fold)."""
    n, L = 48, 180 * 44100
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, 44100, seed0=3000)
    offs, lens = np.arange(n) * L, np.full(n, L)
    got = sdsp.analyze_batch_device(buf.ptr, offs, lens, 44100)
    rig = sdsp.last_key_near(n).copy()
    st = sdsp.stage_times()
    with sdsp.key_cert_fixed():
        got_f = sdsp.analyze_batch_device(buf.ptr, offs, lens, 44100)
        fix = sdsp.last_key_near(n).copy()
    assert all(rig[i] != 0 for i in range(n) if fix[i] != 0), (rig, fix)
    assert st["key_reruns"] == int((rig != 0).sum())
    print(f"rigorous certificate: {int((rig != 0).sum())} of {n} tracks rerun, fixed margins: {int((fix != 0).sum())}")
    xs = [buf.to_host(int(offs[i]), L) for i in range(n)]
    with cf.ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(lambda x: oracle.analyze(x, 44100), xs))
    for i, (rc, ref) in enumerate(refs):
        assert rc == 0, i
        assert got[i]["key"] == ref["key"] and got_f[i]["key"] == ref["key"], i
        assert not parity.diff_results(got[i], ref), (i, parity.diff_results(got[i], ref))
        g, e = parity.result_digest(got[i]), parity.result_digest(ref)
        assert all(g[k] == e[k] for k in g if k not in parity.KEY_ENERGY_FIELDS), i
        if rig[i]:
            assert parity.exact_fraction(got[i], ref, strict=True) == 1.0, i


def test_tail_rerun_in_place_equals_nested(monkeypatch):
    """The last sub-batch's near-decision tracks are rerun in place (Pipeline::rerun_tail: the
    mask completed outside HPCP's band, the exact energy fold, the vote) instead of by a nested
    pipeline from the samples.  With the late key join off (SDSP_NO_KEY_DEFER) the same tracks take
    the nested rerun; every result field must be identical, and so must the rerun count."""
    n, L = 48, 180 * 44100
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, 44100, seed0=3000)
    offs, lens = np.arange(n) * L, np.full(n, L)
    monkeypatch.delenv("SDSP_NO_KEY_DEFER", raising=False)
    got = sdsp.analyze_batch_device(buf.ptr, offs, lens, 44100)
    st = sdsp.stage_times()
    near = sdsp.last_key_near(n).copy()
    monkeypatch.setenv("SDSP_NO_KEY_DEFER", "1")
    ref = sdsp.analyze_batch_device(buf.ptr, offs, lens, 44100)
    st_ref = sdsp.stage_times()
    assert (near != 0).sum() > 0 and st["key_reruns"] == st_ref["key_reruns"] == int((near != 0).sum())
    for i in range(n):
        assert parity.result_digest(got[i]) == parity.result_digest(ref[i]), i
