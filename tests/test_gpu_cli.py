"""The command-line front-ends (stratum-dsp_amd/bin/analyze_file, analyze_batch) on the GPU:
decode -> analyze_audio -> compute_confidence -> the reference examples' output formats
(examples/analyze_file.rs:722-770, examples/analyze_batch.rs:328-380), checked field by field
against the oracle's results run through the host restatement of compute_confidence."""
import json
import os
import subprocess

import numpy as np
import pytest

import host_restate as hr
import oracle
import parity

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "stratum-dsp_amd", "bin")
GOLDEN = os.path.join(ROOT, "tests", "golden")
FIXTURES = ["120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"]


def _expected(path):
    x, sr = parity.load_wav(path)
    st, ref = oracle.analyze(x, sr)
    assert st == 0
    md = ref["metadata"]
    c = hr.compute_confidence(ref["bpm"], ref["bpm_confidence"], ref["key_confidence"], ref["key_clarity"],
                              ref["grid_stability"], md["flags"], md["confidence_warnings"])
    mode, tonic = next(iter(ref["key"].items()))
    key = ["C", "C#", "D", "D#", "E", "F", "F#", "G", "G#", "A", "A#", "B"][tonic % 12] + ("m" if mode == "Minor" else "")
    return ref, c, key


def _f(v, d):
    return f"{float(np.float32(v)):.{d}f}"


@pytest.mark.parametrize("name", FIXTURES)
def test_analyze_file_json(name):
    path = os.path.join(GOLDEN, name)
    out = subprocess.run([os.path.join(BIN, "analyze_file"), path, "--json"], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    ref, c, key = _expected(path)
    lines = out.stdout.splitlines()
    got = json.loads(out.stdout)
    assert lines[1] == f'  "bpm": {_f(ref["bpm"], 2)},'
    assert lines[2] == f'  "bpm_confidence": {_f(c["bpm_confidence"], 2)},'
    assert got["key"] == key
    assert lines[4] == f'  "key_confidence": {_f(c["key_confidence"], 2)},'
    assert lines[5] == f'  "key_clarity": {_f(ref["key_clarity"], 2)},'
    assert lines[6] == f'  "grid_stability": {_f(ref["grid_stability"], 2)},'
    for k in ("tempogram_multi_res_triggered", "tempogram_multi_res_used", "tempogram_percussive_triggered",
              "tempogram_percussive_used"):
        assert got.get(k) == ref["metadata"][k]
    assert "processing_time_ms" in got and lines[-1] == "}"


def test_analyze_file_text_and_flags():
    path = os.path.join(GOLDEN, "120bpm_4bar.wav")
    out = subprocess.run([os.path.join(BIN, "analyze_file"), path, "--no-trim", "--bpm-candidates-top", "5"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("Analysis Results:\n  BPM: ")
    out = subprocess.run([os.path.join(BIN, "analyze_file"), path, "--json", "--bpm-candidates"],
                         capture_output=True, text=True, timeout=300)
    got = json.loads(out.stdout)
    assert got["bpm_candidates"] and all(set(c) == {"bpm", "score", "fft_norm", "autocorr_norm", "selected"}
                                         for c in got["bpm_candidates"])


def test_analyze_batch_jsonl(tmp_path):
    bad = tmp_path / "broken.wav"
    bad.write_bytes(b"RIFF\x04\x00\x00\x00WAVE")
    paths = [os.path.join(GOLDEN, n) for n in FIXTURES] + [str(bad)]
    out = subprocess.run([os.path.join(BIN, "analyze_batch"), "--json", "--jobs", "3"] + paths, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rows = [json.loads(ln) for ln in out.stdout.splitlines()]
    assert [r["file"] for r in rows] == paths
    for p, r in zip(paths[:-1], rows[:-1]):
        ref, c, key = _expected(p)
        assert _f(r["bpm"], 2) == _f(ref["bpm"], 2)
        assert f'{r["bpm_confidence"]:.4f}' == _f(c["bpm_confidence"], 4)
        assert r["key"] == key and f'{r["key_confidence"]:.4f}' == _f(c["key_confidence"], 4)
        assert r["tempogram_multi_res_triggered"] == ref["metadata"]["tempogram_multi_res_triggered"]
    assert rows[-1]["error"].startswith("decode failed:")
    assert "Done: ok=4/5" in out.stderr and "processing_time_ms: mean=" in out.stderr
