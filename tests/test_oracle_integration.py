"""The CPU restatement (oracle/) on the reference's own fixtures (CPU only).

* tests/integration_tests.rs:46-275 — every assertion the reference makes on its WAV fixtures
  (tests/golden/*.wav, copied from the reference's tests/fixtures) holds for the oracle.
* src/lib.rs:100-147 + src/error.rs:24-34 — hard errors and their Display texts.
* tests/golden/oracle_results.json — the oracle's full results (made by
  tests/golden/make_golden.py) stay bit-identical: these are the golden vectors the GPU engine
  is held to.
"""
import json
import sys
import os

import numpy as np
import pytest

import oracle
import parity
import synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIX = ["120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"]


def _run(name):
    x, sr = parity.load_wav(os.path.join(GOLDEN, name))
    st, r = oracle.analyze(x, sr)
    assert st == 0, r
    return r, sr


def test_120bpm_kick():  # integration_tests.rs:46-124
    r, sr = _run("120bpm_4bar.wav")
    md = r["metadata"]
    assert 7.0 < md["duration_seconds"] < 9.0
    assert md["processing_time_ms"] > 0.0 and md["sample_rate"] == sr
    assert r["bpm"] > 0.0
    assert abs(r["bpm"] - 120.0) < 2.0 and r["bpm_confidence"] > 0.0
    b = r["beat_grid"]["beats"]
    assert len(b) >= 4 and 0.0 <= r["grid_stability"] <= 1.0
    assert abs((b[1] - b[0]) - 0.5) < 0.1
    d = r["beat_grid"]["downbeats"]
    if len(d) >= 2:
        assert 1.0 <= d[1] - d[0] <= 4.0


def test_128bpm_kick():  # integration_tests.rs:126-189
    r, _ = _run("128bpm_4bar.wav")
    assert 7.0 < r["metadata"]["duration_seconds"] < 8.0
    assert r["bpm"] > 0.0 and abs(r["bpm"] - 128.0) <= 2.0 and r["bpm_confidence"] > 0.0
    b = r["beat_grid"]["beats"]
    assert len(b) >= 4 and 0.0 <= r["grid_stability"] <= 1.0
    assert abs((b[1] - b[0]) - 60.0 / 128.0) < 0.1


def test_cmajor_scale():  # integration_tests.rs:191-229
    r, _ = _run("cmajor_scale.wav")
    assert r["key"] == {"Major": 0} or r["key_confidence"] < 0.3
    assert 0.0 <= r["key_confidence"] <= 1.0


def test_mixed_silence_trim():  # integration_tests.rs:231-256
    r, _ = _run("mixed_silence.wav")
    assert 4.0 <= r["metadata"]["duration_seconds"] <= 6.0


def test_silent_input_errors():  # integration_tests.rs:258-275
    st, msg = oracle.analyze(np.zeros(44100 * 30, np.float32), 44100)
    assert st == 3 and "silent" in msg
    assert msg == "Processing error: Audio is entirely silent after trimming"


def test_invalid_inputs():  # src/lib.rs:100-110
    st, msg = oracle.analyze(np.zeros(0, np.float32), 44100)
    assert st == 1 and msg == "Invalid input: Empty audio samples"
    st, msg = oracle.analyze(np.ones(100, np.float32), 0)
    assert st == 1 and msg.startswith("Invalid input:")


def _golden():
    with open(os.path.join(GOLDEN, "oracle_results.json")) as f:
        return json.load(f)


def _same(got, want):
    got = dict(got)
    got["metadata"] = {k: v for k, v in got["metadata"].items() if k != "processing_time_ms"}
    assert json.loads(json.dumps(got, sort_keys=True)) == want


@pytest.mark.parametrize("name", FIX)
def test_golden_fixture_results(name):
    r, _ = _run(name)
    _same(r, _golden()["fixtures"][name])


SYNTH_KEYS = [f"{s}:{(30, 30, 45, 20)[s] if s < 4 else (20, 30, 45)[s % 3]}" for s in range(16)]


@pytest.mark.parametrize("key", SYNTH_KEYS)
def test_golden_synthetic_results(key):
    seed, sec = key.split(":")
    x, *_ = synth.make_track(int(seed), seconds=float(sec))
    st, r = oracle.analyze(x, 44100)
    assert st == 0
    _same(r, _golden()["synthetic"][key])


@pytest.mark.parametrize("key", FIX + SYNTH_KEYS)
def test_golden_stage_checksums(key):
    """Per-stage checksums (trim, onset lists, novelty, base tempogram and candidates, escalation,
    beat-grid branches, key arrays) stay identical: the oracle cannot drift stage by stage."""
    sys.path.insert(0, GOLDEN)
    import make_golden

    if key in FIX:
        x, sr = parity.load_wav(os.path.join(GOLDEN, key))
    else:
        seed, sec = key.split(":")
        x, sr = synth.make_track(int(seed), seconds=float(sec))[0], 44100
    got = json.loads(json.dumps(make_golden.stages(x, sr)))
    assert got == _golden()["stages"][key]
