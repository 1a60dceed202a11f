"""debug_track_id diagnostics: the reference prints them to stderr with eprintln!
(src/lib.rs:461-487 base tempogram, 547-573 multi-res decision, 1471-1538 key;
multi_resolution.rs:304-403 candidate lists and GT support, 707-745 folds, 845-857 triplet family).
The engine prints the same blocks per analysed track, in batch order.

Checked here (GPU, stderr captured at the file-descriptor level): every track gets its base block
and key block, escalated tracks their multi-res and decision blocks; the numbers printed agree with
the oracle's trace (base estimate, its candidate support signals, the multi-resolution estimate and
acceptance, the key and its confidence); and switching the dumps on changes no result.
"""
import re

import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu

BPMS = [62.0, 74.0, 184.0, 128.0, 92.0]


def _cfg(base, gt=None):
    base.has_debug_track_id = 1
    base.debug_track_id = 7
    if gt is not None:
        base.has_debug_gt_bpm = 1
        base.debug_gt_bpm = gt
    base.debug_top_n = 4
    return base


def _blocks(text):
    """Split the dump into per-track groups: a group starts at each base block."""
    parts = re.split(r"\n(?==== DEBUG base tempogram)", "\n" + text)
    return [p for p in parts if p.strip()]


def _cand_support(cands, bpm, tol):
    best = np.float32(0.0)
    for c in cands:
        if abs(np.float32(c[0]) - np.float32(bpm)) <= tol:
            best = max(best, np.float32(c[1]))
    return best


def test_debug_dumps(capfd):
    xs = [synth.make_track(900 + k, seconds=40.0, bpm=b)[0] for k, b in enumerate(BPMS)]
    plain = sdsp.analyze_batch(xs, 44100, sdsp.default_config())
    capfd.readouterr()
    got = sdsp.analyze_batch(xs, 44100, _cfg(sdsp.default_config(), gt=120.0))
    err = capfd.readouterr().err
    for a, b in zip(got, plain):
        assert not parity.diff_results(a, b)
    groups = _blocks(err)
    assert len(groups) == len(xs), err[:2000]
    n_mr = 0
    for i, (x, g) in enumerate(zip(xs, groups)):
        st, ref, tr = oracle.analyze(x, 44100, trace=True)
        assert st == 0
        b_bpm, b_conf, b_agree = tr["base"]
        assert "=== DEBUG base tempogram (track_id=7) ===" in g and "GT bpm: 120.000" in g
        amb = bool(tr["ambiguous"])
        assert (f"base_est: bpm={np.float32(b_bpm):.2f} conf={np.float32(b_conf):.4f} agree={b_agree} "
                f"(trap_low={'true' if 55 <= b_bpm <= 80 else 'false'} "
                f"trap_high={'true' if 170 <= b_bpm <= 200 else 'false'} "
                f"ambiguous={'true' if amb else 'false'})") in g, g
        tol = np.float32(2.0)
        cs = tr["base_cands"]
        s_base = _cand_support(cs, b_bpm, tol)
        s_2x = _cand_support(cs, np.float32(b_bpm) * np.float32(2.0), tol)
        s_half = _cand_support(cs, np.float32(b_bpm) * np.float32(0.5), tol)
        assert f"(s_base={s_base:.4f} s_2x={s_2x:.4f} s_half={s_half:.4f})" in g, g
        assert ("NOTE: multi-res not run" in g) == (not amb)
        if tr["ran_mr"] and tr["mr"][0] > 0:
            n_mr += 1
            m_bpm, m_conf, m_agree = tr["mr"]
            assert "=== DEBUG multi-res (track_id=7) ===" in g and "hop=256 top-4:" in g and "hop=1024 top-4:" in g
            assert "Support near GT / family (lookup tol=2.00):" in g
            assert f"mr_est:   bpm={np.float32(m_bpm):.2f} conf={np.float32(m_conf):.4f} agree={m_agree}" in g, g
            used = "true" if tr["used_mr"] else "false"
            assert f"mr_better={used} used_mr={used}" in g
        else:
            assert "=== DEBUG multi-res decision" not in g
        key = ref["key_name"] if "key_name" in ref else None
        assert "=== DEBUG key (track_id=7) ===" in g
        assert f"conf={np.float32(ref['key_confidence']):.4f} clarity={np.float32(ref['key_clarity']):.4f}" in g, g
        if key:
            assert f"key={key} " in g
        m = re.search(r"top_keys: (.*)", g)
        assert m and len(m.group(1).split(", ")) == 3
        m = re.search(r"top_pitch_classes\(weighted\): (.*)", g)
        vals = [float(t.split(":")[1]) for t in m.group(1).split(", ")]
        assert len(vals) == 6 and vals == sorted(vals, reverse=True)
    assert n_mr >= 2, n_mr
