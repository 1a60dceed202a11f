"""ctypes wrapper of the CPU restatement (oracle/build/libsdsp_oracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker — never by the product path (stratum-dsp_amd/).
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "stratum-dsp_amd", "python"))
from sdsp_abi import SdspConfig, SdspResult, result_to_dict  # noqa: E402

LIB_PATH = os.path.join(HERE, "build", "libsdsp_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-j8", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        fp = C.POINTER(C.c_float)
        L.sdsp_oracle_config_default.argtypes = [C.POINTER(SdspConfig)]
        L.sdsp_oracle_analyze.argtypes = [fp, C.c_uint64, C.c_uint32, C.POINTER(SdspConfig), C.POINTER(SdspResult),
                                          C.c_char_p, C.c_uint64]
        L.sdsp_oracle_analyze.restype = C.c_int32
        L.sdsp_oracle_result_free.argtypes = [C.POINTER(SdspResult)]
        L.sdsp_oracle_last_trace_json.restype = C.c_char_p
        L.sdsp_oracle_stft.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint64, fp]
        L.sdsp_oracle_stft.restype = C.c_int64
        L.sdsp_oracle_rfft.argtypes = [fp, C.c_uint64, fp]
        L.sdsp_oracle_fft.argtypes = [fp, C.c_uint64]
        L.sdsp_oracle_novelty_full.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint32, fp]
        L.sdsp_oracle_novelty_full.restype = C.c_int64
        u64p = C.POINTER(C.c_uint64)
        L.sdsp_oracle_vote_onsets.argtypes = [u64p, C.c_uint64] * 4 + [fp, C.c_uint32, C.c_uint32, u64p,
                                                                        C.POINTER(C.c_uint32), fp]
        L.sdsp_oracle_vote_onsets.restype = C.c_int64
        L.sdsp_oracle_key_clarity.argtypes = [fp, C.c_int32]
        L.sdsp_oracle_key_clarity.restype = C.c_float
        L.sdsp_oracle_key_templates.argtypes = [fp]
        L.sdsp_oracle_libm.argtypes = [C.c_int32, fp, fp, fp, C.c_uint64]
        L.sdsp_oracle_find_best.argtypes = [fp, fp, C.c_int32, fp, fp, fp]
        L.sdsp_oracle_find_best.restype = C.c_int32
        L.sdsp_oracle_normalize.argtypes = [C.c_int32, fp, C.c_uint64, C.c_uint32, C.c_char_p, C.c_uint64]
        L.sdsp_oracle_normalize.restype = C.c_int32
        L.sdsp_oracle_hmm_model.argtypes = [C.c_float, fp, fp]
        L.sdsp_oracle_hmm_track.argtypes = [C.c_float, fp, C.c_int32, fp, C.c_int32]
        L.sdsp_oracle_hmm_track.restype = C.c_int32
        L.sdsp_oracle_chroma.argtypes = [C.c_int32, fp, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64,
                                         C.c_int32, C.c_float, C.c_float, fp, C.c_uint64, fp, fp, C.c_uint64]
        L.sdsp_oracle_chroma.restype = C.c_int64
        L.sdsp_oracle_tuning.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.c_float]
        L.sdsp_oracle_tuning.restype = C.c_float
        L.sdsp_oracle_key_hpss.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                                           C.c_uint64, C.c_float]
        L.sdsp_oracle_legacy.argtypes = [C.c_int32, C.POINTER(C.c_uint64), C.c_uint64, C.c_uint32, C.c_uint64,
                                          C.c_float, C.c_float, C.c_float, fp, fp, C.c_uint64, C.c_uint64, fp, fp, fp,
                                          C.POINTER(C.c_uint32), C.c_uint64]
        L.sdsp_oracle_legacy.restype = C.c_int64
        L.sdsp_oracle_hpss.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint64, fp, fp]
        L.sdsp_oracle_hpss.restype = C.c_int32
        L.sdsp_oracle_hpss_onsets.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_float, C.POINTER(C.c_uint64),
                                              C.c_uint64]
        L.sdsp_oracle_hpss_onsets.restype = C.c_int64
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def default_config():
    c = SdspConfig()
    lib().sdsp_oracle_config_default(C.byref(c))
    return c


def analyze(samples, sample_rate=44100, config=None, trace=False):
    """Returns (status, result_dict_or_error_message[, trace_dict])."""
    x = np.ascontiguousarray(samples, dtype=np.float32)
    cfg = config if config is not None else default_config()
    r = SdspResult()
    err = C.create_string_buffer(512)
    st = lib().sdsp_oracle_analyze(_fp(x), x.size, sample_rate, C.byref(cfg), C.byref(r), err, 512)
    tr = json.loads(lib().sdsp_oracle_last_trace_json().decode()) if trace else None
    if st != 0:
        out = (st, err.value.decode())
    else:
        out = (0, result_to_dict(r))
        lib().sdsp_oracle_result_free(C.byref(r))
    return out + ((tr,) if trace else ())


def stft(x, nfft, hop):
    x = np.ascontiguousarray(x, dtype=np.float32)
    if x.size < nfft:
        return np.zeros((0, nfft // 2 + 1), np.float32)
    frames = (x.size - nfft) // hop + 1
    out = np.empty((frames, nfft // 2 + 1), np.float32)
    n = lib().sdsp_oracle_stft(_fp(x), x.size, nfft, hop, _fp(out))
    assert n == frames
    return out


def rfft(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.size // 2 + 1, np.complex64)
    lib().sdsp_oracle_rfft(_fp(x), x.size, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def fft(z):
    z = np.array(z, dtype=np.complex64)
    lib().sdsp_oracle_fft(z.ctypes.data_as(C.POINTER(C.c_float)), z.size)
    return z


def novelty_full(mags, sample_rate=44100):
    m = np.ascontiguousarray(mags, dtype=np.float32)
    out = np.empty(max(m.shape[0], 1), np.float32)
    n = lib().sdsp_oracle_novelty_full(_fp(m), m.shape[0], m.shape[1], sample_rate, _fp(out))
    return out[:n]


def vote_onsets(lists, weights, tol_ms, sample_rate):
    arrs = [np.ascontiguousarray(l, dtype=np.uint64) for l in lists]
    total = sum(a.size for a in arrs) + 1
    t = np.zeros(total, np.uint64)
    v = np.zeros(total, np.uint32)
    cf = np.zeros(total, np.float32)
    w = np.ascontiguousarray(weights, dtype=np.float32)
    args = []
    for a in arrs:
        args += [a.ctypes.data_as(C.POINTER(C.c_uint64)), a.size]
    n = lib().sdsp_oracle_vote_onsets(*args, _fp(w), tol_ms, sample_rate, t.ctypes.data_as(C.POINTER(C.c_uint64)),
                                      v.ctypes.data_as(C.POINTER(C.c_uint32)), _fp(cf))
    if n < 0:
        return int(n)
    return [(int(t[i]), int(v[i]), float(cf[i])) for i in range(n)]


def key_clarity(scores):
    s = np.ascontiguousarray(scores, dtype=np.float32)
    return float(lib().sdsp_oracle_key_clarity(_fp(s), s.size))


def key_templates():
    out = np.empty((24, 12), np.float32)
    lib().sdsp_oracle_key_templates(_fp(out))
    return out


def normalize(x, method, sample_rate=44100):
    """normalization::normalize (lib.rs's fixed config) -> (status, samples or error message)."""
    v = np.array(x, dtype=np.float32)
    err = C.create_string_buffer(256)
    st = lib().sdsp_oracle_normalize(method, _fp(v), v.size, sample_rate, err, 256)
    return (st, v) if st == 0 else (st, err.value.decode())


def libm(op, x, y=None):
    ops = {"ln": 0, "exp": 1, "cos": 2, "log10": 3, "log2": 4, "pow": 5, "sin": 6, "atan2": 7}
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), dtype=np.float32)
    out = np.empty_like(x)
    lib().sdsp_oracle_libm(ops[op], _fp(x), _fp(y), _fp(out), x.size)
    return out


def chroma(mode, spec, sample_rate=44100, fft_size=8192, hop=512, soft=True, sigma=0.5, tuning=0.0, beats=()):
    """Key chroma front-ends on a (frames, bins) magnitude spectrogram -> (chroma (rows, 12), energies).
    mode: "plain" frame_to_chroma_tuned, "hpcp", "logfreq", "beatsync"."""
    m = {"plain": 0, "hpcp": 1, "logfreq": 2, "beatsync": 3}[mode]
    s = np.ascontiguousarray(spec, dtype=np.float32)
    b = np.ascontiguousarray(beats, dtype=np.float32)
    cap = max(s.shape[0], b.size) + 1
    ch = np.zeros((cap, 12), np.float32)
    en = np.zeros(cap, np.float32)
    n = lib().sdsp_oracle_chroma(m, _fp(s), s.shape[0], s.shape[1], sample_rate, fft_size, hop, int(soft),
                                 C.c_float(sigma), C.c_float(tuning), _fp(b), b.size, _fp(ch), _fp(en), cap)
    assert n >= 0
    return ch[:n].copy(), en[:n].copy()


def key_hpss(spec, sample_rate=44100, fft_size=8192, step=4, time_margin=8, freq_margin=8, power=2.0):
    """harmonic_spectrogram_hpss_median_mask over [100, 5000] Hz (src/lib.rs:1014-1024)."""
    s = np.array(spec, dtype=np.float32, order="C")
    lib().sdsp_oracle_key_hpss(_fp(s), s.shape[0], s.shape[1], sample_rate, fft_size, step, time_margin, freq_margin,
                               C.c_float(power))
    return s


def legacy(which, onsets=(), sample_rate=44100, hop=512, min_bpm=40.0, max_bpm=240.0, res=1.0, guardrails=None,
           autocorr=(), comb=()):
    """Legacy BPM estimator pieces (src/features/period): which = "autocorr" | "comb" | "estimate" |
    "merge".  Returns a list of (bpm, confidence, method_agreement), or -(AnalysisError code)."""
    w = {"autocorr": 0, "comb": 1, "estimate": 2, "merge": 3}[which]
    on = np.ascontiguousarray(onsets, dtype=np.uint64)
    cands = list(autocorr) + list(comb)
    ib = np.ascontiguousarray([c[0] for c in cands] or [0.0], dtype=np.float32)
    ic = np.ascontiguousarray([c[1] for c in cands] or [0.0], dtype=np.float32)
    g = None if guardrails is None else np.ascontiguousarray(guardrails, dtype=np.float32)
    cap = 8192
    ob = np.zeros(cap, np.float32)
    oc = np.zeros(cap, np.float32)
    oa = np.zeros(cap, np.uint32)
    n = lib().sdsp_oracle_legacy(w, on.ctypes.data_as(C.POINTER(C.c_uint64)), on.size, sample_rate, hop,
                                 C.c_float(min_bpm), C.c_float(max_bpm), C.c_float(res), _fp(ib), _fp(ic),
                                 len(autocorr), len(comb), _fp(g) if g is not None else None, _fp(ob), _fp(oc),
                                 oa.ctypes.data_as(C.POINTER(C.c_uint32)), cap)
    if n < 0:
        return int(n)
    return [(float(ob[i]), float(oc[i]), int(oa[i])) for i in range(min(n, cap))]


def hpss(spec, margin):
    """hpss_decompose (hpss.rs:71-172) -> (status, harmonic, percussive)."""
    s = np.ascontiguousarray(spec, dtype=np.float32)
    frames = s.shape[0] if s.ndim == 2 else 0
    bins = s.shape[1] if s.ndim == 2 else 0
    h = np.zeros((frames, bins), np.float32)
    p = np.zeros((frames, bins), np.float32)
    st = lib().sdsp_oracle_hpss(_fp(s), frames, bins, margin, _fp(h), _fp(p))
    return st, h, p


def hpss_onsets(perc, pct):
    """detect_hpss_onsets (hpss.rs:275-373) -> onset frame list, or None on Err."""
    s = np.ascontiguousarray(perc, dtype=np.float32)
    frames = s.shape[0] if s.ndim == 2 else 0
    bins = s.shape[1] if s.ndim == 2 else 0
    out = np.zeros(frames + 2, np.uint64)
    n = lib().sdsp_oracle_hpss_onsets(_fp(s), frames, bins, C.c_float(pct), out.ctypes.data_as(C.POINTER(C.c_uint64)),
                                      out.size)
    return None if n < 0 else [int(v) for v in out[:n]]


def tuning(spec, sample_rate=44100, fft_size=8192, frame_step=20, rel_threshold=0.35):
    """estimate_tuning_offset_semitones_from_spectrogram over [80, 2000] Hz (src/lib.rs:1101-1109)."""
    s = np.ascontiguousarray(spec, dtype=np.float32)
    return lib().sdsp_oracle_tuning(_fp(s), s.shape[0], s.shape[1], sample_rate, fft_size, frame_step,
                                    C.c_float(rel_threshold))


def find_best(tempogram):
    """find_best_bpm_fft / find_best_bpm_autocorr on a (bpm, value) list sorted by value desc."""
    b = np.ascontiguousarray([t[0] for t in tempogram], dtype=np.float32)
    v = np.ascontiguousarray([t[1] for t in tempogram], dtype=np.float32)
    ob, ov, oc = C.c_float(), C.c_float(), C.c_float()
    ok = lib().sdsp_oracle_find_best(_fp(b), _fp(v), len(tempogram), C.byref(ob), C.byref(ov), C.byref(oc))
    return (ob.value, ov.value, oc.value) if ok else None


def hmm_model(bpm):
    """(state BPMs, 5x5 transition matrix) of HmmBeatTracker (hmm.rs:165-219)."""
    st = np.empty(5, np.float32)
    tr = np.empty(25, np.float32)
    lib().sdsp_oracle_hmm_model(C.c_float(bpm), _fp(st), _fp(tr))
    return st, tr.reshape(5, 5)


def hmm_track(bpm, onsets_s):
    """HmmBeatTracker::track_beats beat times, or None on Err."""
    on = np.ascontiguousarray(onsets_s, dtype=np.float32)
    cap = 4 * on.size + 64
    out = np.empty(cap, np.float32)
    n = lib().sdsp_oracle_hmm_track(C.c_float(bpm), _fp(on), on.size, _fp(out), cap)
    return None if n < 0 else out[:n].copy()
