"""End-to-end parity of the HIP engine against the CPU restatement (oracle) on the same inputs.

Inputs: the reference's own WAV fixtures (tests/golden/*.wav, copied from
/root/reference/tests/fixtures), seeded synthetic tracks generated on the device (copied back to
the host for the oracle), and edge cases (empty, silent, ultra-short, silence-padded, ragged
batches).  Everything goes through the C ABI (libstratum_hip.so).
"""
import os

import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIXTURES = ["120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"]


def _check(x, sr=44100, label=""):
    st, ref = oracle.analyze(x, sr)
    if st != 0:
        with pytest.raises(sdsp.AnalysisError) as ei:
            sdsp.analyze_audio(x, sr)
        assert ei.value.code == st, (label, ei.value, ref)
        assert str(ei.value) == ref, (label, str(ei.value), ref)
        return None
    got = sdsp.analyze_audio(x, sr)
    bad = parity.diff_results(got, ref)
    assert not bad, f"{label}: {bad}"
    return got, ref


@pytest.mark.parametrize("name", FIXTURES)
def test_reference_fixtures(name):
    x, sr = parity.load_wav(os.path.join(GOLDEN, name))
    got, ref = _check(x, sr, name)
    assert parity.exact_fraction(got, ref) == 1.0, (got, ref)


def test_reference_integration_ranges():
    """tests/integration_tests.rs:46-256 assertions, on the GPU results."""
    x, sr = parity.load_wav(os.path.join(GOLDEN, "120bpm_4bar.wav"))
    r = sdsp.analyze_audio(x, sr)
    assert 7.0 < r["metadata"]["duration_seconds"] < 9.0
    assert abs(r["bpm"] - 120.0) < 2.0 and r["bpm_confidence"] > 0.0
    b = r["beat_grid"]["beats"]
    assert len(b) >= 4 and abs((b[1] - b[0]) - 0.5) < 0.1
    x, sr = parity.load_wav(os.path.join(GOLDEN, "128bpm_4bar.wav"))
    r = sdsp.analyze_audio(x, sr)
    assert 7.0 < r["metadata"]["duration_seconds"] < 8.0
    assert abs(r["bpm"] - 128.0) <= 2.0
    x, sr = parity.load_wav(os.path.join(GOLDEN, "cmajor_scale.wav"))
    r = sdsp.analyze_audio(x, sr)
    assert r["key"] == {"Major": 0} or r["key_confidence"] < 0.3
    x, sr = parity.load_wav(os.path.join(GOLDEN, "mixed_silence.wav"))
    r = sdsp.analyze_audio(x, sr)
    assert 4.0 <= r["metadata"]["duration_seconds"] <= 6.0


def test_errors():
    with pytest.raises(sdsp.AnalysisError) as e:
        sdsp.analyze_audio(np.zeros(0, np.float32), 44100)
    assert e.value.kind == "InvalidInput" and str(e.value) == "Invalid input: Empty audio samples"
    with pytest.raises(sdsp.AnalysisError) as e:
        sdsp.analyze_audio(np.zeros(44100 * 30, np.float32), 44100)
    assert e.value.kind == "ProcessingError" and "silent" in str(e.value)
    with pytest.raises(sdsp.AnalysisError) as e:
        sdsp.analyze_audio(np.ones(100, np.float32), 0)
    assert e.value.kind == "InvalidInput"


@pytest.mark.parametrize("n", [1, 100, 2047, 2048, 2600, 5000, 8191, 8192, 9000, 44100])
def test_short_tracks(n):
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n) * 0.2).astype(np.float32)
    _check(x, 44100, f"short{n}")


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_synthetic_30s(seed):
    x, *_ = synth.make_track(seed, seconds=30.0)
    _check(x, 44100, f"synth{seed}")


def test_silence_padded():
    x, *_ = synth.make_track(11, seconds=20.0, silence_pad=3.0)
    _check(x, 44100, "padded")


def test_ragged_batch_matches_single():
    tracks = [synth.make_track(s, seconds=sec)[0] for s, sec in [(21, 12.0), (22, 31.0), (23, 5.0), (24, 47.5)]]
    tracks.insert(2, np.zeros(0, np.float32))
    res = sdsp.analyze_batch(tracks, 44100)
    for i, (x, r) in enumerate(zip(tracks, res)):
        st, ref = oracle.analyze(x, 44100)
        if st != 0:
            assert isinstance(r, sdsp.AnalysisError) and r.code == st
            continue
        assert not isinstance(r, sdsp.AnalysisError), r
        assert not parity.diff_results(r, ref), (i, parity.diff_results(r, ref))


def test_sub_batches_match_one_batch(monkeypatch):
    """A 1 GB HBM budget splits the batch into several sub-batches (equal shares, ragged
    lengths); every result must equal the single-sub-batch run's."""
    tracks = [synth.make_track(300 + s, seconds=20.0 + 3.0 * (s % 7))[0] for s in range(40)]
    whole = sdsp.analyze_batch(tracks, 44100)
    monkeypatch.setenv("SDSP_HBM_BUDGET_GB", "1")
    split = sdsp.analyze_batch(tracks, 44100)
    for i, (a, b) in enumerate(zip(whole, split)):
        a = {k: v for k, v in a.items() if k != "metadata"} | {"d": a["metadata"]["duration_seconds"]}
        b = {k: v for k, v in b.items() if k != "metadata"} | {"d": b["metadata"]["duration_seconds"]}
        assert a == b, i


def test_host_batch_chunks_match_one_chunk(monkeypatch):
    """sdsp_analyze_batch's chunked work queue (copy of chunk k+1 overlapping the analysis of
    chunk k): 3-track chunks give the same results as one chunk, empty tracks included."""
    tracks = [synth.make_track(700 + s, seconds=8.0 + 2.0 * (s % 5))[0] for s in range(11)]
    tracks.insert(4, np.zeros(0, np.float32))
    whole = sdsp.analyze_batch(tracks, 44100)
    monkeypatch.setenv("SDSP_BATCH_CHUNK_TRACKS", "3")
    split = sdsp.analyze_batch(tracks, 44100)
    for i, (a, b) in enumerate(zip(whole, split)):
        if isinstance(a, sdsp.AnalysisError):
            assert isinstance(b, sdsp.AnalysisError) and a.code == b.code, i
            continue
        a = {k: v for k, v in a.items() if k != "metadata"} | {"d": a["metadata"]["duration_seconds"]}
        b = {k: v for k, v in b.items() if k != "metadata"} | {"d": b["metadata"]["duration_seconds"]}
        assert a == b, i


def test_device_generated_3min_tracks():
    """Device-resident batch (the bench path) on two 3-min synthetic tracks, checked on the host."""
    n, L = 2, 44100 * 180
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, seed0=100)
    res = sdsp.analyze_batch_device(buf.ptr, np.arange(n) * L, np.full(n, L))
    host = buf.to_host()
    for i in range(n):
        st, ref = oracle.analyze(host[i * L:(i + 1) * L], 44100)
        assert st == 0
        assert not parity.diff_results(res[i], ref), (i, parity.diff_results(res[i], ref))


def test_config4_mixed_lengths():
    """BASELINE config 4 shape: device-generated tracks of 30 s to 10 min in one ragged batch
    (frames 2,580 -> 51,676 at 2048/512; FFT-tempogram sizes from 4,096 up to the global-memory
    path), each checked against the oracle."""
    secs = [30, 75, 240, 600]
    xs = []
    for k, sec in enumerate(secs):
        L = 44100 * sec
        buf = sdsp.DeviceBuffer(L)
        sdsp.generate_synthetic(buf.ptr, 1, L, seed0=400 + k)
        xs.append(buf.to_host())
    res = sdsp.analyze_batch(xs, 44100)
    for sec, x, r in zip(secs, xs, res):
        st, ref = oracle.analyze(x, 44100)
        assert st == 0 and not isinstance(r, sdsp.AnalysisError), (sec, r)
        assert not parity.diff_results(r, ref), (sec, parity.diff_results(r, ref))
        assert parity.exact_fraction(r, ref) == 1.0, sec


def test_config5_escalation_heavy():
    """BASELINE config 5 mix (BPMs 1/3 in [55,80], 1/3 in [170,200], 1/3 in [80,170]): the
    multi-resolution escalation runs for most tracks; bpm, confidence and the escalation flags
    must equal the oracle's."""
    n, L = 9, 44100 * 60
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, seed0=500, bpm_mode=1)
    res = sdsp.analyze_batch_device(buf.ptr, np.arange(n) * L, np.full(n, L))
    host = buf.to_host()
    trig = 0
    for i in range(n):
        st, ref = oracle.analyze(host[i * L:(i + 1) * L], 44100)
        assert st == 0
        assert not parity.diff_results(res[i], ref), (i, parity.diff_results(res[i], ref))
        m = res[i]["metadata"]
        assert m["tempogram_multi_res_triggered"] == ref["metadata"]["tempogram_multi_res_triggered"]
        assert m["tempogram_multi_res_used"] == ref["metadata"]["tempogram_multi_res_used"]
        trig += m["tempogram_multi_res_triggered"] is True
    assert trig >= n // 3, trig  # the trap-range thirds escalate


def test_reference_bench_sine():
    """The reference's Criterion workload (benches/audio_analysis_bench.rs:25-29): 30 s of a
    440 Hz sine at 0.5, f32 arithmetic in the bench's order."""
    f32 = np.float32
    i = np.arange(44100 * 30, dtype=np.float32)
    x = (np.sin(i * f32(440.0) * f32(2.0) * f32(np.pi) / f32(44100)) * f32(0.5)).astype(np.float32)
    got, ref = _check(x, 44100, "sine30")
    assert parity.exact_fraction(got, ref) == 1.0


def test_emit_candidates_config():
    x, *_ = synth.make_track(5, seconds=25.0)
    cfg = sdsp.default_config()
    cfg.emit_tempogram_candidates = 1
    got = sdsp.analyze_audio(x, 44100, cfg)
    ocfg = oracle.default_config()
    ocfg.emit_tempogram_candidates = 1
    st, ref = oracle.analyze(x, 44100, ocfg)
    assert st == 0
    assert not parity.diff_results(got, ref)
    gc, rc = got["metadata"]["tempogram_candidates"], ref["metadata"]["tempogram_candidates"]
    assert len(gc) == len(rc)
    for a, b in zip(gc, rc):
        assert abs(a["bpm"] - b["bpm"]) <= 1e-4 and abs(a["score"] - b["score"]) <= 1e-4
        assert a["selected"] == b["selected"]


def _golden():
    import json

    with open(os.path.join(GOLDEN, "oracle_results.json")) as f:
        return json.load(f)


def _strip(r):
    import json

    r = dict(r)
    r["metadata"] = {k: v for k, v in r["metadata"].items() if k != "processing_time_ms"}
    return json.loads(json.dumps(r, sort_keys=True))


@pytest.mark.parametrize("name", FIXTURES)
def test_golden_fixture_vectors(name):
    """Bit-exact against the committed golden vectors (tests/golden/oracle_results.json), the key
    energies' two fields within 1e-4 (parity.KEY_ENERGY_FIELDS)."""
    x, sr = parity.load_wav(os.path.join(GOLDEN, name))
    assert parity.dicts_match(_strip(sdsp.analyze_audio(x, sr)), _golden()["fixtures"][name])


def test_golden_synthetic_vectors():
    g = _golden()["synthetic"]
    keys = sorted(g)
    tracks = []
    for k in keys:
        seed, sec = k.split(":")
        tracks.append(synth.make_track(int(seed), seconds=float(sec))[0])
    for k, r in zip(keys, sdsp.analyze_batch(tracks, 44100)):
        assert parity.dicts_match(_strip(r), g[k]), k
