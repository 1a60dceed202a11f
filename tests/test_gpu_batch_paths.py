"""The batch entry points on real hardware, beyond the per-kernel parity tests (GPU, C ABI).

* sdsp_analyze_batch's multi-device chunk path (the reference's caller-side fan-out,
  examples/analyze_batch.rs:239-268): the devices=(0, 0) test hook maps two workers onto device 0, so
  both copier threads, both copy streams, the slot `ready` events and the shared chunk counter
  run for real on a one-GPU box.  Ragged tracks in 3-track chunks; every result equals the
  oracle's and lands in its own slot; an injected chunk failure (the fail_chunk test hook) marks
  exactly that chunk's tracks.
* A config-2-shaped batch (BASELINE.json configs[1]: 3-min 44.1 kHz tracks) split into >= 3
  sub-batches by SDSP_HBM_BUDGET_GB under the default two-stream schedule: all 64 results
  against the committed oracle digests (tests/golden/config2_oracle.json, made by
  tests/golden/make_config2_golden.py), 8 strided tracks against the oracle live.
* sdsp_analyze_audio from several host threads at once (the reference's API is pure
  and reentrant, src/lib.rs:86-90): each result equals the oracle's.
* A repeated sdsp_analyze_audio call allocates no device memory (the direct one-track path
  reuses the context's buffers).
* Unnormalised int-scale input (enable_normalization = false, samples ~2^23): the STFT
  overflow rule keeps the spectrogram in the reference's range; equal to the oracle.
"""
import concurrent.futures as cf
import ctypes as C
import json
import os

import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config2_oracle.json")


def _ragged_tracks(n, seed0):
    rng = np.random.default_rng(seed0)
    out = []
    for i in range(n):
        sec = float(rng.choice([0.0, 0.05, 3.0, 7.5, 12.0, 21.0]))
        if sec == 0.0:
            out.append(np.zeros(0, np.float32))
            continue
        x, *_ = synth.make_track(seed0 + i, seconds=sec)
        out.append(x)
    return out


def _check_against_oracle(res, tracks):
    for i, (r, x) in enumerate(zip(res, tracks)):
        st, ref = oracle.analyze(x, 44100)
        if st != 0:
            assert isinstance(r, sdsp.AnalysisError) and r.code == st, (i, r)
            continue
        assert not isinstance(r, sdsp.AnalysisError), (i, r)
        assert not parity.diff_results(r, ref), (i, parity.diff_results(r, ref))
        assert parity.exact_fraction(r, ref) == 1.0, i


def test_multidevice_chunk_path_two_workers_on_device0(monkeypatch):
    tracks = _ragged_tracks(40, 5100)
    monkeypatch.setenv("SDSP_BATCH_CHUNK_TRACKS", "3")
    with sdsp.test_hooks(devices=(0, 0)):
        res = sdsp.analyze_batch(tracks)
    assert len(res) == len(tracks)
    _check_against_oracle(res, tracks)


def test_multidevice_chunk_failure_marks_only_its_tracks(monkeypatch):
    tracks = _ragged_tracks(20, 5300)
    monkeypatch.setenv("SDSP_BATCH_CHUNK_TRACKS", "3")
    with sdsp.test_hooks(devices=(0, 0), fail_chunk=2):  # tracks 6, 7, 8
        res = sdsp.analyze_batch(tracks, strict=False)
    for i in (6, 7, 8):
        assert isinstance(res[i], sdsp.AnalysisError) and "injected chunk failure" in str(res[i]), (i, res[i])
    rest = [i for i in range(len(tracks)) if i not in (6, 7, 8)]
    _check_against_oracle([res[i] for i in rest], [tracks[i] for i in rest])
    # the same batch without the failure hook: every track analysed (the pool's slots are reused)
    with sdsp.test_hooks(devices=(0, 0)):
        res2 = sdsp.analyze_batch(tracks)
    _check_against_oracle(res2, tracks)


def test_config2_shaped_sub_batches(monkeypatch):
    with open(GOLD) as f:
        gold = json.load(f)
    n, L = gold["n"], gold["length"]
    buf = sdsp.DeviceBuffer(n * L)
    sdsp.generate_synthetic(buf.ptr, n, L, seed0=gold["seed0"])
    monkeypatch.setenv("SDSP_HBM_BUDGET_GB", "10")  # ~0.5 GB per track: 4 sub-batches
    monkeypatch.delenv("SDSP_SERIAL_STREAMS", raising=False)
    res = sdsp.analyze_batch_device(buf.ptr, np.arange(n) * L, np.full(n, L))
    st = sdsp.stage_times()
    assert st["stft8192_launches"] >= 3, st  # one key STFT launch per sub-batch
    xs = {}
    for i in range(n):
        x = buf.to_host(i * L, L)
        assert parity.samples_digest(x) == gold["tracks"][i]["samples"], i  # the same input
        assert not isinstance(res[i], sdsp.AnalysisError), (i, res[i])
        assert parity.digests_match(parity.result_digest(res[i]), gold["tracks"][i]["result"]), i
        if i % 8 == 3:
            xs[i] = x
    with cf.ThreadPoolExecutor(8) as ex:
        refs = dict(zip(xs, ex.map(lambda x: oracle.analyze(x, 44100), xs.values())))
    for i, (stt, ref) in refs.items():
        assert stt == 0 and parity.exact_fraction(res[i], ref) == 1.0, i


def test_config3_shards_through_eight_workers(monkeypatch):
    """BASELINE config 3 (8192 3-min tracks sharded across 8 GPUs, 1024 per rank: bench.py's
    shard_seed0, seeds 1024 r ..): three tracks from each of the eight shard seed ranges (first,
    middle, last) through sdsp_analyze_batch with an 8-entry device list.  The test build maps
    every entry to device 0, so eight workers, eight copier threads and their copy streams deal
    the 24 tracks out of the shared chunk counter (3-track chunks: one per worker) as the
    reference's caller-side fan-out does (examples/analyze_batch.rs:239-268).  Every result is
    checked against the oracle."""
    L = 180 * 44100
    seeds = [1024 * r + k for r in range(8) for k in (0, 511, 1023)]
    buf = sdsp.DeviceBuffer(L)
    tracks = []
    for s in seeds:
        sdsp.generate_synthetic(buf.ptr, 1, L, seed0=s)
        tracks.append(buf.to_host(0, L))
    monkeypatch.setenv("SDSP_BATCH_CHUNK_TRACKS", "3")
    monkeypatch.delenv("SDSP_SERIAL_STREAMS", raising=False)
    with sdsp.test_hooks(devices=(0,) * 8):
        res = sdsp.analyze_batch(tracks)
    assert len(res) == len(seeds)
    with cf.ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(lambda x: oracle.analyze(x, 44100), tracks))
    for i, ((st, ref), r) in enumerate(zip(refs, res)):
        assert st == 0, (seeds[i], ref)
        assert not isinstance(r, sdsp.AnalysisError), (seeds[i], r)
        assert not parity.diff_results(r, ref), (seeds[i], parity.diff_results(r, ref))
        assert parity.exact_fraction(r, ref) == 1.0, seeds[i]


def test_concurrent_callers():
    tracks = [synth.make_track(5400 + k, seconds=12.0 + 3 * k)[0] for k in range(8)]
    with cf.ThreadPoolExecutor(4) as ex:
        got = list(ex.map(lambda x: sdsp.analyze_audio(x, 44100), tracks))
    _check_against_oracle(got, tracks)


def _alloc_stats():
    L = sdsp.lib()
    f = L.sdsp_debug_alloc_stats
    f.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    n, b = C.c_uint64(), C.c_uint64()
    assert f(C.byref(n), C.byref(b)) == 0
    return n.value, b.value


def test_repeated_analyze_audio_allocates_nothing():
    i = np.arange(44100 * 30, dtype=np.float32)
    f32 = np.float32
    x = (np.sin(i * f32(440.0) * f32(2.0) * f32(np.pi) / f32(44100)) * f32(0.5)).astype(np.float32)
    first = sdsp.analyze_audio(x, 44100)
    a0 = _alloc_stats()
    for _ in range(3):
        again = sdsp.analyze_audio(x, 44100)
        assert parity.result_digest(again) == parity.result_digest(first)
    assert _alloc_stats() == a0
    # and the batch entry point reuses its pooled staging area the same way
    sdsp.analyze_batch([x, x[: 44100 * 10]])
    a1 = _alloc_stats()
    sdsp.analyze_batch([x, x[: 44100 * 10]])
    assert _alloc_stats() == a1


def test_unnormalised_int_scale_input():
    cfg = sdsp.default_config()
    cfg.enable_normalization = 0
    for k in range(3):
        x, *_ = synth.make_track(5500 + k, seconds=20.0)
        x = (x * np.float32(2.0 ** 23)).astype(np.float32)
        got = sdsp.analyze_audio(x, 44100, config=cfg)
        st, ref = oracle.analyze(x, 44100, config=cfg)
        assert st == 0
        assert np.isfinite(got["bpm"]) and np.isfinite(got["key_confidence"])
        assert not parity.diff_results(got, ref), parity.diff_results(got, ref)
        assert parity.exact_fraction(got, ref, cfg=cfg) == 1.0


def test_unnormalised_overflowing_magnitudes():
    """Samples at 2^60 with enable_normalization = false: a tone bin's |X|^2 overflows f32 in the
    reference's own formula (extractor.rs:352), so those magnitudes are +inf.  k_features then
    meets quotients X / max outside its FMA-corrected range (an inf operand) and redoes those
    chunks with the IEEE division; the whole analysis (NaN / inf propagation included) equals the
    oracle's."""
    cfg = sdsp.default_config()
    cfg.enable_normalization = 0
    x, *_ = synth.make_track(5600, seconds=12.0)
    x = (x * np.float32(2.0 ** 60)).astype(np.float32)
    st, ref = oracle.analyze(x, 44100, config=cfg)
    if st != 0:  # the reference fails this input: the engine fails it with the same error
        with pytest.raises(sdsp.AnalysisError) as ei:
            sdsp.analyze_audio(x, 44100, config=cfg)
        assert str(ei.value) == ref, (str(ei.value), ref)
        return
    got = sdsp.analyze_audio(x, 44100, config=cfg)
    assert not parity.diff_results(got, ref), parity.diff_results(got, ref)
