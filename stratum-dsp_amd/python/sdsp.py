"""Python binding of libstratum_hip.so (the MI355X analyze_audio engine).

This is the ctypes stub a Python caller of the reference's API would use: `analyze_audio`
mirrors `stratum_dsp::analyze_audio(samples, sample_rate, AnalysisConfig)` (reference
src/lib.rs:86) and raises `AnalysisError` with the reference's Display text on failure.

There is no CPU fallback: if the HIP library is missing or no GPU is visible, every compute
call raises.
"""
import contextlib
import ctypes as C
import os
import subprocess

import numpy as np

from sdsp_abi import ERROR_NAMES, FLAG_NAMES, SdspConfidence, SdspConfig, SdspResult, SdspStageTimes, result_to_dict

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SDSP_LIB_PATH") or os.path.join(PKG, "lib", "libstratum_hip.so")  # override: layout/ablation builds
# the test build (-DSDSP_TEST_HOOKS): the same library with failure injection and the device
# override compiled in; only test_hooks(fail_chunk=..., devices=...) switches to it
TESTHOOKS_LIB_PATH = os.path.join(PKG, "lib", "libstratum_hip_testhooks.so")
_lib = None
_lib_th = None


class AnalysisError(Exception):
    """AnalysisError (reference src/error.rs:7-34); .kind is the variant name."""

    def __init__(self, code, message):
        super().__init__(message)
        self.code = code
        self.kind = ERROR_NAMES.get(code, "Unknown")


def build():
    subprocess.check_call(["make", "-s", "-j8", "-C", PKG])


def lib():
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH)
    return _lib


def _load(path):
    """ctypes handle of one build of the engine, with the ABI's argument types declared."""
    if True:
        if not os.path.exists(path):
            raise RuntimeError(f"{os.path.basename(path)} not built ({path}); run __graft_entry__.build()")
        L = C.CDLL(path)
        fp = C.POINTER(C.c_float)
        u64p = C.POINTER(C.c_uint64)
        L.sdsp_config_default.argtypes = [C.POINTER(SdspConfig)]
        L.sdsp_version.restype = C.c_char_p
        L.sdsp_analyze_audio.argtypes = [fp, C.c_uint64, C.c_uint32, C.POINTER(SdspConfig), C.POINTER(SdspResult),
                                         C.c_char_p, C.c_uint64]
        L.sdsp_analyze_audio.restype = C.c_int32
        L.sdsp_analyze_batch.argtypes = [C.POINTER(fp), u64p, C.c_uint64, C.c_uint32, C.POINTER(SdspConfig), C.c_uint32,
                                         C.POINTER(SdspResult)]
        L.sdsp_analyze_batch.restype = C.c_int32
        L.sdsp_analyze_batch_device.argtypes = [C.c_void_p, u64p, u64p, C.c_uint64, C.c_uint32, C.POINTER(SdspConfig),
                                                C.c_int32, C.c_void_p, C.POINTER(SdspResult)]
        L.sdsp_analyze_batch_device.restype = C.c_int32
        L.sdsp_analyze_batch_device_ex.argtypes = [C.c_void_p, u64p, u64p, C.c_uint64, C.c_uint32,
                                                   C.POINTER(SdspConfig), C.c_int32, C.c_void_p, C.c_int32,
                                                   C.POINTER(SdspResult)]
        L.sdsp_analyze_batch_device_ex.restype = C.c_int32
        L.sdsp_result_free.argtypes = [C.POINTER(SdspResult)]
        L.sdsp_generate_synthetic.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64, C.c_int32,
                                              C.c_int32, C.c_void_p, fp, C.POINTER(C.c_int32)]
        L.sdsp_generate_synthetic.restype = C.c_int32
        L.sdsp_last_stage_times.argtypes = [C.c_int32, C.POINTER(SdspStageTimes)]
        L.sdsp_last_stage_times.restype = C.c_int32
        L.sdsp_debug_stft.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_float, fp, fp, C.c_int32]
        L.sdsp_debug_stft.restype = C.c_int32
        u64p = C.POINTER(C.c_uint64)
        L.sdsp_debug_frame_rms.argtypes = [fp, C.c_uint64, u64p, u64p, fp, C.c_uint64, C.c_uint64, C.c_uint64,
                                           C.c_int32, fp, C.c_int32]
        L.sdsp_debug_frame_rms.restype = C.c_int32
        L.sdsp_device_count.restype = C.c_int32
        L.sdsp_device_malloc.argtypes = [C.c_int32, C.c_uint64, C.POINTER(C.c_void_p)]
        L.sdsp_device_free.argtypes = [C.c_int32, C.c_void_p]
        L.sdsp_memcpy_h2d.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64]
        L.sdsp_memcpy_d2h.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64]
        L.sdsp_device_synchronize.argtypes = [C.c_int32]
        L.sdsp_compute_confidence.argtypes = [C.POINTER(SdspResult), C.POINTER(SdspConfidence)]
        L.sdsp_key_name.argtypes = [C.c_int32, C.c_uint32, C.c_char_p, C.c_uint64]
        L.sdsp_decode_audio_file.argtypes = [C.c_char_p, C.POINTER(fp), u64p, C.POINTER(C.c_uint32), C.c_char_p,
                                             C.c_uint64]
        L.sdsp_free_samples.argtypes = [fp]
        L.sdsp_free_samples.restype = None
        for f in ("sdsp_device_malloc", "sdsp_device_free", "sdsp_memcpy_h2d", "sdsp_memcpy_d2h",
                  "sdsp_device_synchronize", "sdsp_compute_confidence", "sdsp_key_name", "sdsp_decode_audio_file"):
            getattr(L, f).restype = C.c_int32
        L.sdsp_debug_key_energy_blocked.argtypes = [C.POINTER(SdspConfig), C.c_uint32]
        L.sdsp_debug_key_energy_blocked.restype = C.c_int32
        L.sdsp_debug_set_test_hooks.argtypes = [C.c_int64, C.POINTER(C.c_int32), C.c_uint32, C.c_int32]
        L.sdsp_debug_set_test_hooks.restype = C.c_int32
        return L


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def device_mem_info(device=0):
    """(free, total) bytes of HBM on `device` (sdsp_debug_mem_info)."""
    L = lib()
    f = L.sdsp_debug_mem_info
    f.argtypes = [C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    f.restype = C.c_int32
    fr, to = C.c_uint64(), C.c_uint64()
    if f(device, C.byref(fr), C.byref(to)) != 0:
        raise RuntimeError("sdsp_debug_mem_info failed")
    return fr.value, to.value


@contextlib.contextmanager
def test_hooks(fail_chunk=-1, devices=(), stft_frame_parallel=False):
    """Sets the library's test hooks (include/stratum_hip_debug.h, sdsp_debug_set_test_hooks)
    for the duration of the block, then resets them.  The library reads none of them from the
    environment.  Failure injection and the device override exist only in the test build
    (libstratum_hip_testhooks.so): with either set, every call inside the block goes to it."""
    global _lib, _lib_th, _schedule_set
    test_build = fail_chunk >= 0 or len(devices) > 0
    prev = lib()
    if test_build:
        if _lib_th is None:
            _lib_th = _load(TESTHOOKS_LIB_PATH)
        _lib, _schedule_set = _lib_th, None
    f = _lib.sdsp_debug_set_test_hooks
    dev = (C.c_int32 * max(len(devices), 1))(*devices)
    assert f(fail_chunk, dev if devices else None, len(devices), int(bool(stft_frame_parallel))) == 0
    try:
        yield
    finally:
        f(-1, None, 0, 0)
        if test_build:
            _lib, _schedule_set = prev, None


@contextlib.contextmanager
def key_cert_fixed():
    """sdsp_debug_set_key_cert(1) for the duration of the block: the key vote flags near-decision
    tracks by the fixed round-5 margins alone instead of the rigorous certificate, for
    comparing the two flagged sets."""
    f = lib().sdsp_debug_set_key_cert
    f.argtypes = [C.c_int32]
    f.restype = C.c_int32
    assert f(1) == 0
    try:
        yield
    finally:
        f(0)


def last_key_near(n, device=0):
    """sdsp_debug_last_key_near: per track of the last analysis call on `device`, whether its key
    vote was near an energy-dependent decision (and the track was analysed again exactly): 0, or
    the reason bits (1 within-mode argmax, 2 segment gate, 4 final key gap, 8 weight-sum fallback)."""
    out = np.zeros(max(int(n), 1), np.uint8)
    f = lib().sdsp_debug_last_key_near
    f.argtypes = [C.c_int32, C.c_void_p, C.c_uint64]
    f.restype = C.c_int32
    if f(device, out.ctypes.data, int(n)) != 0:
        raise RuntimeError("sdsp_debug_last_key_near failed")
    return out[: int(n)]


def key_energy_blocked(config=None, sample_rate=44100):
    """sdsp_debug_key_energy_blocked: True when `config` at `sample_rate` takes the default key
    path's block-folded HPCP frame energies (key_confidence / key_clarity re-associated, DESIGN.md
    §2); no device is touched."""
    cfg = config if config is not None else default_config()
    v = lib().sdsp_debug_key_energy_blocked(C.byref(cfg), sample_rate)
    if v < 0:
        raise ValueError("sdsp_debug_key_energy_blocked: bad arguments")
    return bool(v)


_SCHEDULE_ENV = ("SDSP_SERIAL_STREAMS", "SDSP_NO_KEY_DEFER", "SDSP_NO_ROW_REUSE", "SDSP_HOST_TRACE",
                 "SDSP_BATCH_CHUNK_TRACKS", "SDSP_HBM_BUDGET_GB")
_schedule_set = None


def _schedule_from_env():
    """The library reads no environment variable: the test and profiling schedule switches
    (SDSP_SERIAL_STREAMS, SDSP_NO_KEY_DEFER, SDSP_NO_ROW_REUSE, SDSP_HOST_TRACE,
    SDSP_BATCH_CHUNK_TRACKS, SDSP_HBM_BUDGET_GB) are read here, before each analysis call, and passed
    through sdsp_debug_set_schedule (include/stratum_hip_debug.h) when they change."""
    global _schedule_set
    e = os.environ
    knobs = (int(bool(e.get("SDSP_SERIAL_STREAMS"))), int(bool(e.get("SDSP_NO_KEY_DEFER"))),
             int(bool(e.get("SDSP_NO_ROW_REUSE"))), int(bool(e.get("SDSP_HOST_TRACE"))),
             max(int(e.get("SDSP_BATCH_CHUNK_TRACKS") or 0), 0), max(float(e.get("SDSP_HBM_BUDGET_GB") or 0.0), 0.0))
    if knobs == _schedule_set:
        return
    f = lib().sdsp_debug_set_schedule
    f.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_uint64, C.c_double]
    f.restype = C.c_int32
    if f(*knobs) != 0:
        raise RuntimeError("sdsp_debug_set_schedule failed")
    _schedule_set = knobs


def default_config():
    """AnalysisConfig::default() (reference src/config.rs:594-744)."""
    c = SdspConfig()
    lib().sdsp_config_default(C.byref(c))
    return c


def version():
    return lib().sdsp_version().decode()


def analyze_audio(samples, sample_rate=44100, config=None):
    """analyze_audio(samples, sample_rate, config) -> AnalysisResult dict; raises AnalysisError."""
    x = np.ascontiguousarray(samples, dtype=np.float32)
    cfg = config if config is not None else default_config()
    r = SdspResult()
    err = C.create_string_buffer(512)
    _schedule_from_env()
    st = lib().sdsp_analyze_audio(_fp(x), x.size, sample_rate, C.byref(cfg), C.byref(r), err, 512)
    if st != 0:
        raise AnalysisError(st, err.value.decode())
    try:
        return result_to_dict(r)
    finally:
        lib().sdsp_result_free(C.byref(r))


def _batch_error(outs, n, what):
    """Whole-batch failure: the first per-track message, and free whatever was filled."""
    msg = outs[0].error_message.decode() if n > 0 and outs[0].error_message[0:1] != b"\0" else ""
    for i in range(n):
        lib().sdsp_result_free(C.byref(outs[i]))
    return f"{what}: {msg}" if msg else what


def analyze_batch(tracks, sample_rate=44100, config=None, device_mask=0, strict=True):
    """Batch form: list of per-track results; failed tracks come back as AnalysisError objects.
    strict: raise when the call as a whole reports a failure (a failed chunk); otherwise return
    the per-track results, the failed chunk's tracks as AnalysisError."""
    arrs = [np.ascontiguousarray(t, dtype=np.float32) for t in tracks]
    n = len(arrs)
    ptrs = (C.POINTER(C.c_float) * n)(*[_fp(a) for a in arrs])
    lens = np.array([a.size for a in arrs], dtype=np.uint64)
    outs = (SdspResult * n)()
    cfg = config if config is not None else default_config()
    _schedule_from_env()
    st = lib().sdsp_analyze_batch(ptrs, lens.ctypes.data_as(C.POINTER(C.c_uint64)), n, sample_rate, C.byref(cfg),
                                  device_mask, outs)
    if st != 0 and strict:
        raise AnalysisError(st, _batch_error(outs, n, "batch failed"))
    res = []
    for i in range(n):
        if outs[i].status != 0:
            res.append(AnalysisError(outs[i].status, outs[i].error_message.decode()))
        else:
            res.append(result_to_dict(outs[i]))
        lib().sdsp_result_free(C.byref(outs[i]))
    return res


def compute_confidence(result):
    """compute_confidence (src/analysis/confidence.rs:121) through the C ABI, on an
    AnalysisResult dict (as analyze_audio returns).  Returns the AnalysisConfidence fields plus
    the confidence_level() string (confidence.rs:218-228)."""
    r = SdspResult()
    r.bpm = result["bpm"]
    r.bpm_confidence = result["bpm_confidence"]
    r.key_confidence = result["key_confidence"]
    r.key_clarity = result["key_clarity"]
    r.grid_stability = result["grid_stability"]
    md = result.get("metadata", {})
    r.flags = sum(1 << FLAG_NAMES.index(f) for f in set(md.get("flags", [])))
    warns = [w.encode() for w in md.get("confidence_warnings", [])]
    arr = (C.c_char_p * max(len(warns), 1))(*warns)
    r.warnings = C.cast(arr, C.POINTER(C.c_char_p))
    r.n_warnings = len(warns)
    out = SdspConfidence()
    if lib().sdsp_compute_confidence(C.byref(r), C.byref(out)) != 0:
        raise AnalysisError(1, "Invalid input: compute_confidence")
    overall = out.overall_confidence
    level = "High" if overall >= 0.7 else "Low" if overall < 0.5 else "Medium"
    return {"bpm_confidence": out.bpm_confidence, "key_confidence": out.key_confidence,
            "grid_stability": out.grid_stability, "overall_confidence": overall,
            "flags": [FLAG_NAMES[out.flag_list[i]] for i in range(out.n_flags)], "confidence_level": level}


def decode_audio_file(path):
    """The decode front-end (sdsp_decode_audio_file): RIFF/WAVE or FLAC -> (mono float32 array, sample_rate),
    converted as examples/analyze_file.rs:25-180 does.  Raises AnalysisError(DecodingError)."""
    p = C.POINTER(C.c_float)()
    n = C.c_uint64()
    sr = C.c_uint32()
    err = C.create_string_buffer(512)
    st = lib().sdsp_decode_audio_file(os.fsencode(path), C.byref(p), C.byref(n), C.byref(sr), err, 512)
    if st != 0:
        raise AnalysisError(st, "Decoding error: " + err.value.decode(errors="replace"))
    try:
        x = np.ctypeslib.as_array(p, shape=(n.value,)).copy() if n.value else np.zeros(0, np.float32)
    finally:
        lib().sdsp_free_samples(p)
    return x, sr.value


class ResultBatch:
    """The C-ABI result array of one batch call, kept as native structs (no per-track Python
    objects are built until asked for).  Index it for AnalysisResult dicts / AnalysisError."""

    def __init__(self, outs, n):
        self._outs = outs
        self.n = n
        self.status = [outs[i].status for i in range(n)]

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        o = self._outs[i]
        if o.status != 0:
            return AnalysisError(o.status, o.error_message.decode())
        return result_to_dict(o)

    def count(self, field, value=1):
        """How many successful tracks have the native result field == value (e.g.
        tempogram_multi_res_triggered), without building result dicts."""
        return sum(1 for i in range(self.n) if self.status[i] == 0 and getattr(self._outs[i], field) == value)

    def free(self):
        if self._outs is not None:
            for i in range(self.n):
                lib().sdsp_result_free(C.byref(self._outs[i]))
            self._outs = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


STAGES_FULL = 0
STAGES_BPM_ONLY = 1  # stages a1-a19 (src/lib.rs:86-910): no key path, no beat grid


def analyze_batch_device(d_ptr, offsets, lens, sample_rate=44100, config=None, device=0, stream=None, raw=False,
                         stages=STAGES_FULL):
    """Tracks already resident in HBM (d_ptr: device address).  Returns a list of results
    (dicts / AnalysisError), or with raw=True the native ResultBatch.  stages=STAGES_BPM_ONLY runs
    the tempo path alone (sdsp_analyze_batch_device_ex)."""
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    n = ln.size
    outs = (SdspResult * n)()
    cfg = config if config is not None else default_config()
    _schedule_from_env()
    st = lib().sdsp_analyze_batch_device_ex(C.c_void_p(d_ptr), offs.ctypes.data_as(C.POINTER(C.c_uint64)),
                                            ln.ctypes.data_as(C.POINTER(C.c_uint64)), n, sample_rate, C.byref(cfg),
                                            device, C.c_void_p(stream or 0), stages, outs)
    if st != 0:
        raise AnalysisError(st, _batch_error(outs, n, "device batch failed"))
    batch = ResultBatch(outs, n)
    if raw:
        return batch
    res = [batch[i] for i in range(n)]
    batch.free()
    return res


def generate_synthetic(d_ptr, n_tracks, length, sample_rate=44100, seed0=0, bpm_mode=0, device=0, stream=None):
    bpm = np.zeros(n_tracks, np.float32)
    key = np.zeros(n_tracks, np.int32)
    st = lib().sdsp_generate_synthetic(C.c_void_p(d_ptr), n_tracks, length, sample_rate, seed0, bpm_mode, device,
                                       C.c_void_p(stream or 0), _fp(bpm), key.ctypes.data_as(C.POINTER(C.c_int32)))
    if st != 0:
        raise AnalysisError(st, "synthetic generation failed")
    return bpm, key


def stage_times(device=0):
    t = SdspStageTimes()
    lib().sdsp_last_stage_times(device, C.byref(t))
    return {k: getattr(t, k) for k, _ in SdspStageTimes._fields_}


class DeviceBuffer:
    """A float32 buffer in HBM owned through the engine's own HIP runtime."""

    def __init__(self, n_floats, device=0):
        self.device = device
        self.n = int(n_floats)
        p = C.c_void_p()
        if lib().sdsp_device_malloc(device, self.n * 4, C.byref(p)) != 0:
            raise MemoryError(f"sdsp_device_malloc({self.n * 4} bytes) failed")
        self.ptr = p.value

    def to_host(self, start=0, count=None):
        count = self.n - start if count is None else count
        out = np.empty(count, np.float32)
        if lib().sdsp_memcpy_d2h(self.device, out.ctypes.data, self.ptr + 4 * start, 4 * count) != 0:
            raise RuntimeError("sdsp_memcpy_d2h failed")
        return out

    def from_host(self, arr, start=0):
        a = np.ascontiguousarray(arr, dtype=np.float32)
        if lib().sdsp_memcpy_h2d(self.device, self.ptr + 4 * start, a.ctypes.data, 4 * a.size) != 0:
            raise RuntimeError("sdsp_memcpy_h2d failed")

    def free(self):
        if self.ptr:
            lib().sdsp_device_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_count():
    return int(lib().sdsp_device_count())


def synchronize(device=0):
    if lib().sdsp_device_synchronize(device) != 0:
        raise RuntimeError("sdsp_device_synchronize failed")


def debug_frame_rms(tracks, gains, fs, hop, per_frame=False, device=0):
    """Frame RMS of each track (silence-trimming framing), concatenated over tracks."""
    arrs = [np.ascontiguousarray(t, dtype=np.float32) for t in tracks]
    lens = np.array([a.size for a in arrs], np.uint64)
    offs = np.zeros(len(arrs), np.uint64)
    if len(arrs) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    x = np.concatenate(arrs) if arrs else np.zeros(0, np.float32)
    frames = sum(((int(n) - fs) // hop + 1) if n >= fs else (1 if n > 0 else 0) for n in lens)
    out = np.empty(max(frames, 1), np.float32)
    g = np.ascontiguousarray(gains, dtype=np.float32)
    u64p = C.POINTER(C.c_uint64)
    st = lib().sdsp_debug_frame_rms(_fp(x), x.size, offs.ctypes.data_as(u64p), lens.ctypes.data_as(u64p), _fp(g),
                                    len(arrs), fs, hop, 1 if per_frame else 0, _fp(out), device)
    if st != 0:
        raise AnalysisError(st, "debug_frame_rms failed")
    return out[:frames]


def debug_stft(x, nfft, hop, gain=1.0, device=0):
    x = np.ascontiguousarray(x, dtype=np.float32)
    frames = (x.size - nfft) // hop + 1
    out = np.empty((frames, nfft // 2 + 1), np.float32)
    fmax = np.empty(frames, np.float32)
    st = lib().sdsp_debug_stft(_fp(x), x.size, nfft, hop, gain, _fp(out), _fp(fmax), device)
    if st != 0:
        raise AnalysisError(st, "debug_stft failed")
    return out, fmax
