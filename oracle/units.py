"""Unit-level bindings of the CPU restatement (the "unit probes" sections of oracle/o_*.cpp).

TEST INFRASTRUCTURE: imported only by tests/ (tests/test_oracle_units_*.py restate the
reference's own #[test] functions against these).  Each function is named after the reference
function it exposes and raises AnalysisError(code, message) where the reference returns Err.
"""
import ctypes as C

import numpy as np

import oracle

fp = C.POINTER(C.c_float)
u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)

ERRORS = {1: "InvalidInput", 2: "DecodingError", 3: "ProcessingError", 4: "NotImplemented", 5: "NumericalError"}


class AnalysisError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code
        self.kind = ERRORS.get(code, str(code))


_L = None


def lib():
    global _L
    if _L is None:
        L = oracle.lib()
        L.sdsp_oracle_probe_error.restype = C.c_char_p
        L.sdsp_oracle_energy_flux_onsets.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_float, u64p, C.c_uint64]
        L.sdsp_oracle_energy_flux_onsets.restype = C.c_int64
        L.sdsp_oracle_spectral_flux_onsets.argtypes = [fp, C.c_uint64, C.c_uint64, u64p, C.c_float, u64p, C.c_uint64]
        L.sdsp_oracle_spectral_flux_onsets.restype = C.c_int64
        L.sdsp_oracle_hfc_onsets.argtypes = [fp, C.c_uint64, C.c_uint64, u64p, C.c_uint32, C.c_float, u64p, C.c_uint64]
        L.sdsp_oracle_hfc_onsets.restype = C.c_int64
        L.sdsp_oracle_detect_and_trim.argtypes = [fp, C.c_uint64, C.c_uint32, C.c_float, C.c_uint32, C.c_uint64, u64p,
                                                  u64p, C.c_uint64]
        L.sdsp_oracle_detect_and_trim.restype = C.c_int64
        L.sdsp_oracle_novelty.argtypes = [C.c_int32, fp, C.c_uint64, C.c_uint64, u64p, C.c_uint32, C.c_uint64, fp]
        L.sdsp_oracle_novelty.restype = C.c_int64
        L.sdsp_oracle_combined_novelty.argtypes = [fp, C.c_uint64, fp, C.c_uint64, fp, C.c_uint64, C.c_float, C.c_float,
                                                   C.c_float, C.c_uint64, C.c_uint64, fp]
        L.sdsp_oracle_combined_novelty.restype = C.c_int64
        L.sdsp_oracle_tempogram.argtypes = [C.c_int32, fp, C.c_uint64, C.c_uint32, C.c_uint32, C.c_float, C.c_float,
                                            C.c_float, fp, fp, C.c_uint64]
        L.sdsp_oracle_tempogram.restype = C.c_int64
        L.sdsp_oracle_tempogram_estimate.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_float,
                                                     C.c_float, C.c_float, fp]
        L.sdsp_oracle_tempogram_estimate.restype = C.c_int32
        L.sdsp_oracle_multi_resolution_analysis.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_uint32, C.c_float, C.c_float,
                                                            C.c_float, fp]
        L.sdsp_oracle_multi_resolution_analysis.restype = C.c_int32
        L.sdsp_oracle_beat_grid.argtypes = [C.c_float, C.c_float, fp, C.c_uint64, C.c_uint32, fp, fp, C.c_uint64, u64p, fp]
        L.sdsp_oracle_beat_grid.restype = C.c_int32
        L.sdsp_oracle_downbeats.argtypes = [fp, C.c_uint64, C.c_float, C.c_uint32, fp]
        L.sdsp_oracle_downbeats.restype = C.c_int64
        L.sdsp_oracle_grid_stability.argtypes = [fp, C.c_uint64, C.c_float, fp]
        L.sdsp_oracle_grid_stability.restype = C.c_int32
        L.sdsp_oracle_tempo_variations.argtypes = [fp, C.c_uint64, C.c_float, fp, C.c_uint64]
        L.sdsp_oracle_tempo_variations.restype = C.c_int64
        L.sdsp_oracle_bayes.argtypes = [C.c_int32, C.c_float, C.c_float, fp, C.c_uint64, C.c_float, fp, C.c_uint64]
        L.sdsp_oracle_bayes.restype = C.c_int64
        L.sdsp_oracle_time_signature.argtypes = [fp, C.c_uint64, C.c_float, u32p, fp]
        L.sdsp_oracle_time_signature.restype = C.c_int32
        L.sdsp_oracle_detect_key.argtypes = [fp, C.c_uint64, C.c_uint64, fp, C.c_uint64, i32p, fp, fp, i32p]
        L.sdsp_oracle_detect_key.restype = C.c_int32
        L.sdsp_oracle_smooth_chroma.argtypes = [fp, C.c_uint64, C.c_uint64, C.c_int32, fp]
        L.sdsp_oracle_dot.argtypes = [fp, fp, C.c_uint64]
        L.sdsp_oracle_dot.restype = C.c_float
        _L = L
    return _L


def _check(rc):
    if rc < 0:
        raise AnalysisError(-rc, lib().sdsp_oracle_probe_error().decode())
    return rc


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _p(a):
    return a.ctypes.data_as(fp) if a.size else C.cast(C.c_void_p(0), fp)


def _spec(spec):
    """A list of frames (possibly ragged, as the reference's Vec<Vec<f32>>) -> flat, frames,
    bins, row lengths.  Ragged rows are zero-padded; the probe rejects them like the reference."""
    rows = [np.asarray(r, dtype=np.float32) for r in spec]
    frames = len(rows)
    lens = np.array([len(r) for r in rows], dtype=np.uint64)
    bins = int(lens.max()) if frames else 0
    flat = np.zeros((frames, bins), dtype=np.float32)
    for i, r in enumerate(rows):
        flat[i, :len(r)] = r
    return np.ascontiguousarray(flat.ravel()), frames, bins, lens


def _u64(a):
    return a.ctypes.data_as(u64p) if a.size else C.cast(C.c_void_p(0), u64p)


def _list_call(fn, *args, cap=1 << 16):
    out = np.zeros(cap, dtype=np.uint64)
    n = _check(fn(*args, _u64(out), cap))
    return [int(v) for v in out[:n]]


# ---- onsets / preprocessing ----
def detect_energy_flux_onsets(samples, frame_size, hop_size, threshold_db):
    x = _f32(samples)
    return _list_call(lib().sdsp_oracle_energy_flux_onsets, _p(x), x.size, frame_size, hop_size, threshold_db)


def detect_spectral_flux_onsets(spec, percentile):
    flat, fr, b, lens = _spec(spec)
    return _list_call(lib().sdsp_oracle_spectral_flux_onsets, _p(flat), fr, b, _u64(lens), percentile)


def detect_hfc_onsets(spec, sample_rate, percentile):
    flat, fr, b, lens = _spec(spec)
    return _list_call(lib().sdsp_oracle_hfc_onsets, _p(flat), fr, b, _u64(lens), sample_rate, percentile)


def detect_and_trim(samples, sample_rate, threshold_db=-40.0, min_duration_ms=500, frame_size=2048):
    """SilenceDetector::default() = (-40 dB, 500 ms, 2048).  Returns (trimmed samples, silence map)."""
    x = _f32(samples)
    trim = np.zeros(2, dtype=np.uint64)
    cap = 4096
    reg = np.zeros(2 * cap, dtype=np.uint64)
    n = _check(lib().sdsp_oracle_detect_and_trim(_p(x), x.size, sample_rate, threshold_db, min_duration_ms, frame_size,
                                                 _u64(trim), _u64(reg), cap))
    return x[int(trim[0]):int(trim[1])], [(int(reg[2 * i]), int(reg[2 * i + 1])) for i in range(n)]


# ---- novelty / tempograms ----
def _novelty(kind, spec, sample_rate=44100, k=4):
    flat, fr, b, lens = _spec(spec)
    out = np.zeros(max(fr, 1), dtype=np.float32)
    n = _check(lib().sdsp_oracle_novelty(kind, _p(flat), fr, b, _u64(lens), sample_rate, k, _p(out)))
    return out[:n]


def spectral_flux_novelty(spec):
    return _novelty(0, spec)


def energy_flux_novelty(spec):
    return _novelty(1, spec)


def hfc_novelty(spec, sample_rate):
    return _novelty(2, spec, sample_rate)


def superflux_novelty(spec, max_filter_bins):
    return _novelty(3, spec, k=max_filter_bins)


def combined_novelty(spectral, energy, hfc, params=(0.5, 0.3, 0.2, 16, 5)):
    s, e, h = _f32(spectral), _f32(energy), _f32(hfc)
    out = np.zeros(max(s.size, e.size, h.size, 1), dtype=np.float32)
    n = _check(lib().sdsp_oracle_combined_novelty(_p(s), s.size, _p(e), e.size, _p(h), h.size, *params, _p(out)))
    return out[:n]


def _tempogram(kind, novelty, sr, hop, lo, hi, res):
    x = _f32(novelty)
    cap = 1 << 16
    b, v = np.zeros(cap, np.float32), np.zeros(cap, np.float32)
    n = _check(lib().sdsp_oracle_tempogram(kind, _p(x), x.size, sr, hop, lo, hi, res, _p(b), _p(v), cap))
    return list(zip(b[:n].tolist(), v[:n].tolist()))


def fft_tempogram(novelty, sample_rate, hop_size, min_bpm, max_bpm):
    return _tempogram(0, novelty, sample_rate, hop_size, min_bpm, max_bpm, 1.0)


def autocorrelation_tempogram(novelty, sample_rate, hop_size, min_bpm, max_bpm, bpm_resolution):
    return _tempogram(1, novelty, sample_rate, hop_size, min_bpm, max_bpm, bpm_resolution)


def find_best_bpm(tempogram):
    """find_best_bpm_fft / find_best_bpm_autocorr: (bpm, value, confidence) or None."""
    if not tempogram:
        return None
    return oracle.find_best(tempogram)


def estimate_bpm_tempogram(spec, sample_rate, hop_size, min_bpm, max_bpm, bpm_resolution):
    flat, fr, b, _ = _spec(spec)
    out = np.zeros(3, np.float32)
    _check(lib().sdsp_oracle_tempogram_estimate(_p(flat), fr, b, sample_rate, hop_size, min_bpm, max_bpm,
                                                bpm_resolution, _p(out)))
    return float(out[0]), float(out[1]), int(out[2])


def multi_resolution_analysis(spec, sample_rate, base_hop_size, min_bpm, max_bpm, bpm_resolution):
    flat, fr, b, _ = _spec(spec)
    out = np.zeros(3, np.float32)
    _check(lib().sdsp_oracle_multi_resolution_analysis(_p(flat), fr, b, sample_rate, min_bpm, max_bpm, bpm_resolution,
                                                       _p(out)))
    return float(out[0]), float(out[1]), int(out[2])


# ---- beat tracking ----
def generate_beat_grid(bpm, bpm_confidence, onsets_s, sample_rate):
    """(beats, downbeats, bars, stability); AnalysisError where the reference returns Err."""
    on = _f32(onsets_s)
    cap = 1 << 16
    b, d = np.zeros(cap, np.float32), np.zeros(cap, np.float32)
    counts = np.zeros(2, np.uint64)
    st = C.c_float(0)
    rc = lib().sdsp_oracle_beat_grid(bpm, bpm_confidence, _p(on), on.size, sample_rate, _p(b), _p(d), cap, _u64(counts),
                                     C.byref(st))
    if rc != 0:
        raise AnalysisError(1, "generate_beat_grid failed")
    beats, downs = b[:int(counts[0])].tolist(), d[:int(counts[1])].tolist()
    return beats, downs, list(downs), st.value


def detect_downbeats(beats, bpm, beats_per_bar=4):
    x = _f32(beats)
    out = np.zeros(max(x.size, 1), np.float32)
    n = _check(lib().sdsp_oracle_downbeats(_p(x), x.size, bpm, beats_per_bar, _p(out)))
    return out[:n].tolist()


def calculate_grid_stability(times, bpm):
    x = _f32(times)
    v = C.c_float(0)
    _check(lib().sdsp_oracle_grid_stability(_p(x), x.size, bpm, C.byref(v)))
    return v.value


def detect_tempo_variations(beats, nominal_bpm):
    """[(start, end, bpm, confidence, is_variable)]"""
    x = _f32(beats)
    cap = 4096
    out = np.zeros(5 * cap, np.float32)
    n = _check(lib().sdsp_oracle_tempo_variations(_p(x), x.size, nominal_bpm, _p(out), cap))
    return [(float(out[5 * i]), float(out[5 * i + 1]), float(out[5 * i + 2]), float(out[5 * i + 3]),
             bool(out[5 * i + 4])) for i in range(n)]


def has_tempo_variation(segments):
    return any(s[4] for s in segments)  # tempo_variation.rs:225-227


class BayesianBeatTracker:
    """bayesian.rs:77-272; every call rebuilds the tracker from (bpm, confidence) like new()."""

    def __init__(self, initial_bpm, initial_confidence):
        self.bpm0, self.conf0 = float(initial_bpm), float(initial_confidence)
        out = np.zeros(64, np.float32)
        n = _check(lib().sdsp_oracle_bayes(3, self.bpm0, self.conf0, _p(np.zeros(0, np.float32)), 0, 0.0, _p(out), 64))
        self.current_bpm, self.current_confidence = float(out[0]), float(out[1])
        self.history = out[2:2 + n].tolist()

    def _op(self, op, onsets=(), x=0.0, cap=4096):
        on = _f32(onsets)
        out = np.zeros(cap, np.float32)
        n = _check(lib().sdsp_oracle_bayes(op, self.bpm0, self.conf0, _p(on), on.size, x, _p(out), cap))
        return n, out

    def generate_bpm_candidates(self):
        n, out = self._op(0)
        return out[:n].tolist()

    def compute_likelihood(self, onsets, bpm):
        return float(self._op(1, onsets, bpm)[1][0])

    def compute_prior(self, bpm):
        return float(self._op(2, (), bpm)[1][0])

    def update_with_onsets(self, onsets, sample_rate=44100):
        n, out = self._op(4, onsets)
        self.current_bpm, self.current_confidence = float(out[0]), float(out[1])
        self.history = out[2:2 + n].tolist()
        return self.current_bpm, self.current_confidence


def detect_time_signature(beats, bpm):
    x = _f32(beats)
    bpb, conf = C.c_uint32(0), C.c_float(0)
    _check(lib().sdsp_oracle_time_signature(_p(x), x.size, bpm, C.byref(bpb), C.byref(conf)))
    return bpb.value, conf.value


# ---- key ----
def detect_key_weighted(chroma_vectors, weights=None):
    """(key index mode*12+tonic, confidence, all_scores [(key, score)] sorted, top_keys)"""
    rows = [list(r) for r in chroma_vectors]
    dims = len(rows[0]) if rows else 12
    if any(len(r) != dims for r in rows):
        dims = -1  # ragged: rejected like the reference's per-vector check
    flat = _f32([v for r in rows for v in r]) if dims == 12 else np.zeros(0, np.float32)
    w = _f32(weights) if weights is not None else None
    key, conf = C.c_int32(0), C.c_float(0)
    sc, ks = np.zeros(24, np.float32), np.zeros(24, np.int32)
    _check(lib().sdsp_oracle_detect_key(_p(flat), len(rows), dims if dims > 0 else 0, _p(w) if w is not None else None,
                                        w.size if w is not None else 0, C.byref(key), C.byref(conf), _p(sc),
                                        ks.ctypes.data_as(i32p)))
    all_scores = list(zip(ks.tolist(), sc.tolist()))
    return key.value, conf.value, all_scores, all_scores[:3]


def detect_key(chroma_vectors):
    return detect_key_weighted(chroma_vectors, None)


def smooth_chroma(chroma_vectors, window_size, average=False):
    x = _f32(chroma_vectors).reshape(-1)
    frames = x.size // 12
    out = np.zeros(x.size, np.float32)
    lib().sdsp_oracle_smooth_chroma(_p(x), frames, window_size, 1 if average else 0, _p(out))
    return out.reshape(frames, 12)


def smooth_chroma_average(chroma_vectors, window_size):
    return smooth_chroma(chroma_vectors, window_size, average=True)


def dot_product(a, b):
    x, y = _f32(a), _f32(b)
    return lib().sdsp_oracle_dot(_p(x), _p(y), min(x.size, y.size))


def compute_key_clarity(scores):
    return oracle.key_clarity([s for _, s in scores]) if scores else 0.0
