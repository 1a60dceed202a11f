"""Independent float64 restatement of the tempo and beat-grid stages (SURVEY §8a rows a10-a16 and
a20-a23), written from the reference Rust, not from oracle/ (C++).  TEST INFRASTRUCTURE: it is a
second reading of the reference that tests/test_ref64.py compares with the CPU restatement, so a
misreading shared by the oracle and the HIP kernels (which are bit-identical to it) shows up here.

Rules of the restatement:
- continuous quantities (sums, powers, means, products) are float64 and vectorised, so they carry
  none of the f32 fold order the oracle and kernels reproduce;
- discrete parameters the reference computes in f32 and then rounds or truncates (mel band
  edges) are computed in f32 the same way;
- sorts are stable where the reference's are; max_by keeps the last maximum.

Reference files (all under /root/reference/src):
  features/period/novelty.rs:62-190, 336-986       novelty curves, mel filterbank, conditioning
  features/period/tempogram_fft.rs:78-236          FFT tempogram, find_best_bpm_fft
  features/period/tempogram_autocorr.rs:79-222     autocorrelation tempogram
  features/period/tempogram.rs:255-775             estimate_bpm_tempogram_impl (band fusion)
  features/beat_tracking/mod.rs:108-485            generate_beat_grid, downbeats, stability
  features/beat_tracking/hmm.rs:121-441            HMM beat tracker
  features/beat_tracking/tempo_variation.rs:95-227 tempo segments
  features/beat_tracking/bayesian.rs:77-272        Bayesian tempo update
  features/beat_tracking/time_signature.rs:90-199  time signature
"""
import math

import numpy as np

EPS = 1e-10
f32 = np.float32

# AnalysisConfig::default() tempogram settings (config.rs:594-744, src/lib.rs:343-369)
BAND_DEFAULT = dict(enabled=True, low_max_hz=200.0, mid_max_hz=2000.0, high_max_hz=8000.0, w_full=0.40, w_low=0.25,
                    w_mid=0.20, w_high=0.15, seed_only=True, support_threshold=0.25, consensus_bonus=0.08,
                    enable_mel=True, mel_n_mels=40, mel_fmin_hz=30.0, mel_fmax_hz=8000.0, mel_max_filter_bins=2,
                    w_mel=0.15, nw=(0.30, 0.35, 0.35), local_mean=16, smooth=5, superflux_k=4)


def normalize_peak64(x, headroom_db=1.0):
    """normalize_peak in float64 (src/preprocessing/normalization.rs:262-322, src/lib.rs:116-127):
    gain = min(10^(-headroom/20) / peak, 1 / peak) for peak > 1e-10, else the signal unchanged.
    NaN samples are ignored by the peak, as f32::max does."""
    x = np.asarray(x, np.float64)
    a = np.abs(x[np.isfinite(x) | np.isinf(x)])
    peak = float(a.max()) if a.size else 0.0
    if not peak > 1e-10:
        return x
    return x * min(10.0 ** (-headroom_db / 20.0) / peak, 1.0 / peak)


def stft64(x, frame_size=2048, hop=512):
    """compute_stft in float64 with numpy's FFT (src/features/chroma/extractor.rs:301-359):
    frames at multiples of hop while a whole frame fits, the symmetric Hann window
    0.5 (1 - cos(2 pi i / (N - 1))), |rfft| of each windowed frame.  Independent of the CPU
    restatement's FFT and libm (include/sdsp_fft_spec.h, sdsp_libm.h)."""
    x = np.asarray(x, np.float64)
    n = x.size
    if n < frame_size:
        return np.zeros((0, frame_size // 2 + 1))
    nf = (n - frame_size) // hop + 1
    i = np.arange(frame_size)
    w = 0.5 * (1.0 - np.cos(2.0 * np.pi * i / (frame_size - 1)))
    idx = np.arange(nf)[:, None] * hop + i[None, :]
    return np.abs(np.fft.rfft(x[idx] * w, axis=1))


def _normalize(v):
    mx = max(float(v.max()), 0.0) if v.size else 0.0
    return v / mx if mx > EPS else v


def _window_max(P, k):
    """max over columns [b-k, b+k] of each row, from 0 (every input is >= 0, so 0-padding is exact)."""
    F, B = P.shape
    pad = np.zeros((F, B + 2 * k))
    pad[:, k:k + B] = P
    out = np.zeros((F, B))
    for j in range(2 * k + 1):
        out = np.maximum(out, pad[:, j:j + B])
    return out


# ---- novelty.rs ----
def superflux_band(L, k, start, end):
    """superflux_novelty(_band) on ln(1 + max(X, 0)) frames L (novelty.rs:336-455)."""
    F, B = L.shape
    if F < 2:
        return np.zeros(0)
    s, e = min(start, B), min(end, B)
    if e <= s + 1:
        return np.zeros(0)
    k = max(k, 1)
    band = L[:, s:e]
    pm = _window_max(band[:-1], k)
    d = np.maximum(band[1:] - pm, 0.0)
    return _normalize(np.sqrt((d * d).sum(axis=1)))


def scalar_flux(v):
    if v.size < 2:
        return np.zeros(0)
    return _normalize(np.maximum(np.diff(v), 0.0))


def energy_band(M, start, end):
    """energy_flux_novelty(_band) (novelty.rs:477-545, 612-665)."""
    B = M.shape[1]
    s, e = min(start, B), min(end, B)
    if M.shape[0] < 2 or e <= s + 1:
        return np.zeros(0)
    return scalar_flux((M[:, s:e] ** 2).sum(axis=1))


def hfc_band(M, start, end):
    """hfc_novelty(_band) (novelty.rs:687-836): sum_k k |X_k|^2 with absolute bin index k."""
    B = M.shape[1]
    s, e = min(start, B), min(end, B)
    if M.shape[0] < 2 or e <= s + 1:
        return np.zeros(0)
    k = np.arange(s, e, dtype=np.float64)
    return scalar_flux((M[:, s:e] ** 2 * k).sum(axis=1))


def _round_half_away(x):
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def mel_weights(sr, n_bins, n_mels, fmin_hz, fmax_hz):
    """MelFilterbank::new (novelty.rs:71-172): band edges in f32 as the reference rounds them;
    returns the n_bins x n_mels triangle weight matrix (float64)."""
    n_mels = max(n_mels, 4)
    nyq = f32(sr) * f32(0.5)
    fmin = min(max(f32(fmin_hz), f32(0.0)), max(nyq, f32(1.0)))
    fmax = f32(fmax_hz)
    if not (np.isfinite(fmax) and fmax > 0):
        fmax = nyq
    fmax = min(max(fmax, f32(fmin + f32(1.0))), nyq)
    fres = f32(sr) / f32((n_bins - 1) * 2)
    mel = lambda f: f32(2595.0) * f32(np.log10(f32(f32(1.0) + f32(f / f32(700.0)))))
    inv_mel = lambda m: f32(700.0) * f32(f32(np.power(f32(10.0), f32(m / f32(2595.0)))) - f32(1.0))
    mmin, mmax = mel(fmin), mel(fmax)
    step = f32((mmax - mmin) / f32(n_mels + 1))
    pts = [min(max(_round_half_away(float(f32(inv_mel(f32(mmin + f32(step * f32(i)))) / fres))), 0), n_bins - 1)
           for i in range(n_mels + 2)]
    for i in range(1, len(pts)):
        if pts[i] <= pts[i - 1]:
            pts[i] = min(pts[i - 1] + 1, n_bins - 1)
    W = np.zeros((n_bins, n_mels))
    for m in range(n_mels):
        l, c, r = pts[m], pts[m + 1], pts[m + 2]
        if not (l < c < r):
            continue
        for b in range(l, c + 1):
            if b != l:
                W[b, m] += (b - l) / (c - l)
        for b in range(c, r + 1):
            if b != r:
                W[b, m] += (r - b) / (r - c)
    return W


def mel_superflux(M, L, sr, n_mels, fmin, fmax, k):
    """mel_superflux_novelty (novelty.rs:553-609)."""
    if M.shape[0] < 2:
        return np.zeros(0)
    mel = L @ mel_weights(sr, M.shape[1], n_mels, fmin, fmax)
    k = max(k, 1)
    pm = _window_max(mel[:-1], k)
    d = np.maximum(mel[1:] - pm, 0.0)
    return _normalize(np.sqrt((d * d).sum(axis=1)))


def _box_mean(x, window):
    half = max(window, 1) // 2
    n = x.size
    c = np.concatenate([[0.0], np.cumsum(x)])
    i = np.arange(n)
    s, e = np.maximum(i - half, 0), np.minimum(i + half + 1, n)
    return (c[e] - c[s]) / (e - s)


def combine(s, e, h, ws, we, wh, lmw, smw):
    """combined_novelty_with_params (novelty.rs:874-986)."""
    n = min(s.size, e.size, h.size)
    if n == 0:
        return np.zeros(0)
    ws, we, wh = max(ws, 0.0), max(we, 0.0), max(wh, 0.0)
    c = (s[:n] * ws + e[:n] * we + h[:n] * wh) / max(ws + we + wh, EPS)
    c = _normalize(c)
    if lmw > 1:
        c = np.maximum(c - _box_mean(c, lmw), 0.0)
    if smw > 1 and c.size >= 3:
        c = _box_mean(c, smw)
    return _normalize(c)


# ---- tempograms ----
def fft_tempogram(nov, sr, hop, lo, hi):
    """tempogram_fft.rs:78-192: [(bpm, power)] sorted by power, stable."""
    n = nov.size
    P = 1 << max(n - 1, 0).bit_length()
    w = 0.5 * (1.0 - np.cos(2.0 * np.pi * np.arange(n) / (n - 1))) if n > 1 else np.ones(1)
    X = np.fft.rfft((nov - nov.mean()) * w, P)
    power = X.real ** 2 + X.imag ** 2
    # bin BPMs are discrete values the reference computes in f32 (:111, 163-173): the same here
    fres = f32(f32(f32(sr) / f32(hop)) / f32(P))
    bpm = ((np.arange(P // 2 + 1).astype(np.float32) * fres) * f32(60.0)).astype(np.float64)
    keep = (bpm >= lo) & (bpm <= hi)
    b, p = bpm[keep], power[keep]
    order = np.argsort(-p, kind="stable")
    return b[order], p[order]


def acf_tempogram(nov, sr, hop, lo, hi, res):
    """tempogram_autocorr.rs:79-178: strength(bpm) = mean of n_i n_{i+lag}, lag = trunc(frames/beat)."""
    frame_rate = sr / hop
    grid, g = [], f32(lo)
    while g <= f32(hi):  # the reference's f32 BPM accumulator
        grid.append(float(g))
        g = f32(g + f32(res))
    bpm = np.array(grid)
    n = nov.size
    st = np.zeros(bpm.size)
    for i, b in enumerate(bpm):
        lag = int(frame_rate / (b / 60.0))
        if lag < n:
            st[i] = float(np.dot(nov[:n - lag], nov[lag:])) / (n - lag)
    order = np.argsort(-st, kind="stable")
    return bpm[order], st[order]


def find_best(tg):
    b, v = tg
    if b.size == 0:
        return None
    if b.size > 1:
        conf = min(max(max(v[0] - v[1], 0.0) / v[0], 0.0), 1.0) if v[0] > EPS else 0.0
    else:
        conf = 0.5
    return float(b[0]), float(v[0]), conf


LOOKUP_TIE = 2e-4  # BPM: the reference's f32 BPM values are this close to their float64 ones


def _lookup(tg, bpm, tol, tie=None):
    """lookup_nearest (tempogram.rs:517-529): the first of the nearest entries within tol.  A
    candidate that sits (within f32 BPM rounding) midway between two entries, e.g. 1.5 x an odd
    FFT bin, has its lookup decided by rounding: tie[0] is then set."""
    b, v = tg
    if b.size == 0:
        return 0.0
    d = np.abs(b - bpm)
    ok = np.nonzero(d <= tol)[0]
    if ok.size == 0:
        return 0.0
    if tie is not None and ok.size > 1:
        dd = np.sort(d[ok])
        tie[0] |= bool(dd[1] - dd[0] < LOOKUP_TIE)
    return float(v[ok[np.argmin(d[ok])]])


def novelty_full(M, band=BAND_DEFAULT):
    L = np.log1p(np.maximum(M, 0.0))
    B = M.shape[1]
    return combine(superflux_band(L, band["superflux_k"], 0, B), energy_band(M, 0, B), hfc_band(M, 0, B), *band["nw"],
                   band["local_mean"], band["smooth"])


def estimate_bpm_tempogram(M, sr, hop, lo, hi, res, band=BAND_DEFAULT):
    """estimate_bpm_tempogram_impl (tempogram.rs:255-775) with a band configuration.
    Returns (bpm, confidence, agreement, scored) with scored = [(bpm, score, fft_norm, ac_norm)]."""
    F, nb = M.shape
    L = np.log1p(np.maximum(M, 0.0))
    fres = f32(sr) / f32(max((nb - 1) * 2, 2))

    def hz_to_bin(hz):
        if not np.isfinite(hz) or hz <= 0:
            return 0
        return min(max(_round_half_away(float(f32(f32(hz) / fres))), 0), nb - 1)

    nw, lmw, smw, k = band["nw"], band["local_mean"], band["smooth"], band["superflux_k"]
    full = combine(superflux_band(L, k, 0, nb), energy_band(M, 0, nb), hfc_band(M, 0, nb), *nw, lmw, smw)
    if full.size == 0:
        raise ValueError("Novelty curve is empty after extraction")

    def variant(name, w, nov):
        ft, ac = fft_tempogram(nov, sr, hop, lo, hi), acf_tempogram(nov, sr, hop, lo, hi, res)
        return dict(name=name, w=w, fft=ft, ac=ac, max_fft=max(ft[1][0] if ft[1].size else 1.0, 1e-12),
                    max_ac=max(ac[1][0] if ac[1].size else 1.0, 1e-12))

    seeds = [variant("full", band["w_full"], full)]
    fft_best, ac_best = find_best(seeds[0]["fft"]), find_best(seeds[0]["ac"])
    if band["enabled"]:
        b0 = min(1, nb - 1)
        bl = max(hz_to_bin(band["low_max_hz"]), b0)
        bm = max(hz_to_bin(band["mid_max_hz"]), bl + 1)
        bh = max(hz_to_bin(band["high_max_hz"]), bm + 1) if band["high_max_hz"] > 0 else nb
        bh = min(bh, nb)
        for name, s, e, w in (("low", b0, bl, band["w_low"]), ("mid", bl, bm, band["w_mid"]),
                              ("high", bm, bh, band["w_high"])):
            if not (np.isfinite(w) and w > 0) or e <= s + 1:
                continue
            nov = combine(superflux_band(L, k, s, e), energy_band(M, s, e), hfc_band(M, s, e), *nw, lmw, smw)
            if nov.size:
                seeds.append(variant(name, w, nov))
    if band["enable_mel"]:
        mc = mel_superflux(M, L, sr, band["mel_n_mels"], band["mel_fmin_hz"], band["mel_fmax_hz"],
                           band["mel_max_filter_bins"])
        if mc.size:
            seeds.append(variant("mel", band["w_mel"], mc))
    score_v = [v for v in seeds if v["name"] == "full"] if band["seed_only"] else seeds
    support = min(max(band["support_threshold"], 0.0), 1.0)
    bonus = max(band["consensus_bonus"], 0.0)
    w_sum = max(sum(max(v["w"], 0.0) for v in score_v), 1e-6)
    seed_bpms = []
    for v in seeds:
        seed_bpms += list(v["fft"][0][:8]) + list(v["ac"][0][:8])
    if fft_best and fft_best[0] > 0:
        seed_bpms.append(fft_best[0])
    if ac_best and ac_best[0] > 0:
        seed_bpms.append(ac_best[0])
    # candidate BPMs: f32 products with the f32 folding factors (tempogram.rs:551-558)
    facs = [f32(1.0), f32(0.5), f32(2.0), f32(1.0) / f32(3.0), f32(3.0), f32(2.0) / f32(3.0), f32(3.0) / f32(2.0)]
    cands = sorted(x for b in seed_bpms for f in facs
                   for x in [float(f32(f32(b) * f))] if np.isfinite(x) and lo <= x <= hi)
    uniq = []
    for b in cands:
        if uniq and abs(b - uniq[-1]) < 0.75:
            continue
        uniq.append(b)
    ac_tol = max(res, 0.5)
    bonus_on = bonus > 0 and (band["enabled"] or band["enable_mel"])
    scored, lookup_ties = [], set()
    for bpm in uniq:
        fa = aa = 0.0
        tie = [False]
        for v in score_v:
            if v["w"] <= 0:
                continue
            fa += v["w"] * min(max(_lookup(v["fft"], bpm, 0.75, tie) / v["max_fft"], 0.0), 1.0)
            aa += v["w"] * min(max(_lookup(v["ac"], bpm, ac_tol, tie) / v["max_ac"], 0.0), 1.0)
        if tie[0]:
            lookup_ties.add(bpm)
        fn, an = min(max(fa / w_sum, 0.0), 1.0), min(max(aa / w_sum, 0.0), 1.0)
        score = 0.55 * an + 0.45 * fn
        if bonus_on:
            sb = 0
            for v in seeds:
                if v["name"] == "full":
                    continue
                sf = min(max(_lookup(v["fft"], bpm, 0.75) / v["max_fft"], 0.0), 1.0)
                sa = min(max(_lookup(v["ac"], bpm, ac_tol) / v["max_ac"], 0.0), 1.0)
                sb += max(sf, sa) >= support
            if sb >= 2:
                score *= 1.0 + bonus * (sb - 1)
        if bpm > 180.0:
            score *= 0.80
        elif bpm < 60.0:
            score *= 0.90
        scored.append((bpm, score, fn, an))
    scored.sort(key=lambda c: -c[1])  # stable
    best = scored[0]
    if best[0] > 180.0:
        folded = best[0] / 2.0
        if lo <= folded <= hi:
            for c in scored:
                if abs(c[0] - folded) < 0.75:
                    if not ((best[3] + 1e-6) / (c[3] + 1e-6) > 2.0 and (best[2] + 1e-6) / (c[2] + 1e-6) > 2.0):
                        best = c
                    break
    conf = 0.0
    if best[1] > 1e-12:
        second = scored[1][1] if len(scored) > 1 else 0.0
        conf = min(max(max(best[1] - second, 0.0) / best[1], 0.0), 1.0)
    agree = int(bool(fft_best) and fft_best[0] > 0 and abs(fft_best[0] - best[0]) < 2.0)
    agree += int(bool(ac_best) and ac_best[0] > 0 and abs(ac_best[0] - best[0]) < 2.0)
    estimate_bpm_tempogram.lookup_ties = lookup_ties  # candidates whose score f32 rounding decides
    return best[0], conf, agree, scored


# ---- beat tracking ----
SIGMA_E = 0.05 / 2.0  # hmm.rs:55-58


def _nearest_dist(on, t):
    return np.min(np.abs(on[None, :] - np.asarray(t)[:, None]), axis=1)


def hmm_track(bpm, on):
    """HmmBeatTracker::track_beats (hmm.rs:121-441).  The emission is the same for every state, so
    the Viterbi path does not select the beats; they are the frames whose emission exceeds 0.1."""
    if bpm <= EPS or bpm > 300.0 or on.size == 0:
        return None
    # the frame times are the reference's f32 values start + t * (60 / bpm): segment membership
    # (tempo_variation.rs:155-160, mod.rs:164-171) compares them with f32 bounds exactly
    interval = f32(f32(60.0) / f32(bpm))
    on32 = on.astype(np.float32)
    nf = int(math.ceil(float(f32(f32(on32[-1] - on32[0]) / interval)))) + 1
    t = (on32[0] + (np.arange(nf, dtype=np.float32) * interval).astype(np.float32)).astype(np.float32).astype(np.float64)
    d = _nearest_dist(on, t)
    emis = np.exp(-(d * d) / (2.0 * SIGMA_E * SIGMA_E))
    keep = emis > 0.1
    align = np.where(d < 0.05, 1.0 - d / 0.05, 0.0)
    conf = np.minimum(emis * 0.7 + align * 0.3, 1.0)
    return list(zip(t[keep].tolist(), conf[keep].tolist()))


def tempo_segments(beats, nominal):
    """detect_tempo_variations (tempo_variation.rs:95-227): (start, end, bpm, conf, variable)."""
    if len(beats) < 4:
        return [(beats[0] if beats else 0.0, beats[-1] if beats else 0.0, nominal, 0.5, False)]
    b = np.asarray(beats)
    total = f32(f32(b[-1]) - f32(b[0]))  # segment bounds in f32 as the reference computes them
    if total < 2.0:
        return [(b[0], b[-1], nominal, 0.8, False)]
    seg = min(max(f32(total / f32(4.0)), f32(4.0)), f32(8.0))
    step = f32(seg - f32(seg * f32(0.5)))
    cur, segs = f32(b[0]), []
    while cur < b[-1]:
        end = min(f32(cur + seg), f32(b[-1]))
        sb = b[(b >= cur) & (b <= end)]
        if sb.size >= 3:
            iv = np.diff(sb)
            iv = iv[iv > 0]
            if iv.size:
                mean = iv.mean()
                cv = iv.std() / mean if mean > EPS else 0.0
                segs.append((cur, end, 60.0 / mean if mean > EPS else nominal, max(1.0 - min(cv / 0.3, 1.0), 0.0),
                             cv > 0.15))
        cur = f32(cur + step)
    return segs or [(b[0], b[-1], nominal, 0.8, False)]


TIE = 1e-5  # relative margin below which f32 rounding, not the algorithm, decides a comparison


def bayes_update(state, on, ties=None):
    """BayesianBeatTracker::update_with_onsets (bayesian.rs:104-181): state = [bpm, conf]."""
    lo_, hi_ = max(state[0] - 5.0, 60.0), min(state[0] + 5.0, 180.0)
    best_bpm, best_l = state[0], 0.0
    liks = []
    c = lo_
    while c <= hi_:
        bi = 60.0 / c
        idx = np.array([_round_half_away((o - on[0]) / bi) for o in on])
        d = np.abs(on - (on[0] + idx * bi))
        lik = math.exp(float(np.mean(-(d * d) / (2.0 * 0.05 * 0.05))))
        liks.append(lik)
        if lik > best_l:
            best_l, best_bpm = lik, c
        c += 0.5
    if ties is not None and len(liks) > 1:
        top = sorted(liks, reverse=True)
        if top[0] > 0 and (top[0] - top[1]) / top[0] < TIE:
            ties.append(("bayes", best_bpm))
    ch = abs(best_bpm - state[0])
    pen = 1.0 if ch < 1.0 else (0.8 if ch < 3.0 else 0.5)
    state[0], state[1] = best_bpm, min(best_l * pen, 1.0)
    return best_bpm


def time_signature(beats, bpm, ties=None):
    """detect_time_signature (time_signature.rs:90-199): beats per bar (max_by: last maximum)."""
    if len(beats) < 8:
        return 4
    iv = np.diff(np.asarray(beats))
    iv = iv[iv > 0]
    if iv.size == 0:
        return 4
    mean = iv.mean()

    def score(bpb):
        if iv.size < bpb:
            return 0.0
        d = np.abs(iv[:-bpb] - iv[bpb:])
        if d.size == 0:
            return 0.0
        ac = float(np.mean(1.0 / (1.0 + d / mean)))
        cv = iv.std() / mean if mean > EPS else 1.0
        return min(ac * 0.7 + (1.0 / (1.0 + cv)) * 0.3, 1.0)

    scores = {4: score(4), 3: score(3), 6: score(6)}
    best, bs = 4, scores[4]
    for bpb in (3, 6):
        if not scores[bpb] < bs:
            best, bs = bpb, scores[bpb]
    if ties is not None:
        near = [b for b, v in scores.items() if bs - v <= TIE * max(bs, 1e-12)]
        if len(near) > 1:
            ties.append(("time_signature", tuple(sorted(near))))
    return best


def generate_beat_grid(bpm, conf, onsets_s):
    """generate_beat_grid (beat_tracking/mod.rs:108-247) -> (beats, downbeats, stability, diag) or
    None where the reference returns Err (src/lib.rs maps that to an empty grid)."""
    if bpm <= 0.0 or bpm > 300.0 or len(onsets_s) == 0:
        return None
    # onset times are the reference's f32 seconds (src/lib.rs:913-920), compared with f32 bounds
    on = np.sort(np.asarray(onsets_s, dtype=np.float32).astype(np.float64), kind="stable")
    pos = hmm_track(bpm, on)
    if not pos:
        return None
    segs = tempo_segments([p[0] for p in pos], bpm)
    ties = []
    diag = {"variable": any(s[4] for s in segs), "refined": False, "ties": ties, "hmm_beats": [p[0] for p in pos]}
    if diag["variable"]:
        refined, state = [], [bpm, min(max(conf, 0.0), 1.0)]
        for s in segs:
            if s[4]:
                so = on[(on >= s[0]) & (on <= s[1])]
                if so.size:
                    ub = bayes_update(state, so, ties)
                    sb = hmm_track(ub, so)
                    if sb:
                        refined += sb
            else:
                refined += [p for p in pos if s[0] <= p[0] <= s[1]]
        if refined:
            refined.sort(key=lambda p: p[0])
            pos = refined
            diag["refined"] = True
    times = [p[0] for p in pos]
    bpb = time_signature(times, bpm, ties)
    diag["beats_per_bar"] = bpb
    beats = sorted(times)
    bar = (60.0 / bpm) * bpb
    downs = [beats[0]]
    for t in beats[1:]:
        if abs(t - (downs[-1] + bar)) <= bar * 0.1:
            downs.append(t)
    stab = 0.0
    iv = np.diff(np.asarray(times))
    iv = iv[iv > 0]
    if len(times) >= 2 and iv.size and iv.mean() > 1e-10:
        stab = 1.0 / (1.0 + iv.std() / iv.mean())
    return beats, downs, stab, diag


# ---- multi-resolution escalation (a17, a18) ----
# AnalysisConfig::default() (config.rs:610-618, 653, 665)
MR_DEFAULT = dict(top_k=25, w512=0.45, w256=0.35, w1024=0.20, dt512=0.92, margin=0.08, human_prior=False,
                  base_top_n=25)
SCORE_TIE = 1e-5  # score / ratio comparisons closer than this may be decided by the reference's f32 rounding
#                   (f32 and float64 candidate scores differ by < 4e-6: tests/test_ref64_multires.py)


def _near(a, b, eps):
    """a and b differ, by less than eps: the reference's f32 values may order them either way.  Equal
    float64 values are not near ties: they come from exactly representable operands (integer BPM
    grids, halves, zero scores), which f32 holds exactly too."""
    return 0.0 < abs(a - b) < eps


class Ties(list):
    """Comparisons whose outcome f32 rounding decides, as (tag, a, b)."""

    def ge(self, tag, a, b, eps=SCORE_TIE):
        if _near(a, b, eps):
            self.append((tag, a, b))
        return a >= b

    def gt(self, tag, a, b, eps=SCORE_TIE):
        if _near(a, b, eps):
            self.append((tag, a, b))
        return a > b


def cand_lookup(cands, bpm, tol, ties=None, tag="lookup"):
    """lookup_nearest over a candidate list (multi_resolution.rs:282-293): the score of the first
    strictly nearest candidate within tol, else 0.  Candidate BPMs are the reference's f32 values
    (discrete), and the distance is the reference's f32 |c - bpm|, so the pick is the reference's
    own; only an exactly equal distance to two candidates whose list order (by score) is itself a
    near tie is left to f32 rounding."""
    best_d, best_s, best_i, eq = math.inf, 0.0, -1, []
    for i, c in enumerate(cands):
        d = float(abs(f32(c[0]) - f32(bpm)))
        if d <= tol:
            if d < best_d:
                best_d, best_s, best_i, eq = d, c[1], i, []
            elif d == best_d:
                eq.append(i)
    if ties is not None:
        for i in eq:
            if cands[i][1] != best_s and _near(cands[i][1], best_s, SCORE_TIE):
                ties.append((tag + "-order", best_s, cands[i][1]))
    return best_s


def escalation_gate(bpm, conf, agree, cands, res=1.0, ties=None):
    """The ambiguity gate of src/lib.rs:412-457 on the base hop-512 estimate and its candidate list
    (top base_top_n).  Returns (ambiguous, trap_low, trap_high)."""
    ties = Ties() if ties is None else ties
    trap_low = 55.0 <= bpm <= 80.0
    trap_high = 170.0 <= bpm <= 200.0
    tol = max(2.0, res)

    def support(b):  # cand_support (:420-432): the maximum score within tol (f32 distances)
        best = 0.0
        for c in cands:
            if float(abs(f32(c[0]) - f32(b))) <= tol:
                best = max(best, c[1])
        return best

    s_base, s_2x, s_half = support(bpm), support(bpm * 2.0), support(bpm * 0.5)  # x2, x0.5: exact in f32
    family = (s_2x > 0.0 and ties.ge("gate-2x", s_2x, s_base * 0.90)) or \
             (s_half > 0.0 and ties.ge("gate-half", s_half, s_base * 0.90))
    fold_into_trap = 170.0 <= bpm * 2.0 <= 200.0
    weak = agree == 0 or conf < 0.06
    if _near(conf, 0.06, SCORE_TIE):
        ties.append(("gate-weak", conf, 0.06))
    return bool(trap_low or trap_high or family or (weak and fold_into_trap)), trap_low, trap_high


def beat_contrast(nov, sr, hop, bpm, ties=None):
    """beat_contrast_score (multi_resolution.rs:580-678), float64."""
    n = nov.size
    if n < 16 or not (math.isfinite(bpm) and bpm > 0):
        return 0.0
    fpb = 60.0 * sr / (bpm * hop)
    if not math.isfinite(fpb) or fpb < 3.0:
        return 0.0
    if ties is not None and _near(fpb - math.floor(fpb), 0.5, 1e-5):
        ties.append(("mr-period-round", fpb, 0.5))  # f32 frames-per-beat rounds either way
    period = _round_half_away(fpb)
    if not 3 <= period <= 512:
        return 0.0
    w = 2
    pad = np.concatenate([np.zeros(w), nov, np.zeros(w)])  # every value is >= 0: 0-padding is exact
    wmax = np.max(np.stack([pad[j:j + n] for j in range(2 * w + 1)]), axis=0)
    total = max(float(nov.sum()), 1e-6)
    best = -1e9
    for ph in range(period):
        idx = np.arange(ph, n, period)
        bm = float(wmax[idx].mean()) if idx.size else 0.0
        hm = tm = 0.0
        if period >= 6:
            j = idx + period // 2
            j = j[j < n]
            hm = float(wmax[j].mean()) if j.size else 0.0
        if period >= 9:
            j1, j2 = idx + period // 3, idx + (2 * period) // 3
            # the reference interleaves the 1/3 and 2/3 windows per beat; a mean does not care
            jj = np.concatenate([j1[j1 < n], j2[j2 < n]])
            tm = float(wmax[jj].mean()) if jj.size else 0.0
        contrast = bm - 0.60 * hm - 0.40 * tm
        best = max(best, min(max(contrast / max(total / n, 1e-6), -10.0), 10.0))
    return best


def multi_resolution(x, sr, stft, frame_size=2048, lo=40.0, hi=240.0, res=1.0, mr=MR_DEFAULT, band=BAND_DEFAULT,
                     ties=None):
    """multi_resolution_tempogram_from_samples (multi_resolution.rs:205-901) on the trimmed,
    normalised samples x.  stft(x, nfft, hop) supplies the magnitudes (the spec-pinned STFT).
    Returns (bpm, confidence, agreement)."""
    ties = Ties() if ties is None else ties
    if x.size < frame_size:
        raise ValueError("Audio too short for STFT")
    top_k = max(mr["top_k"], 1)
    aux_k = min(max(top_k * 4, 25), 200)
    tol = max(2.0, res)
    spec = {h: stft(x, frame_size, h).astype(np.float64) for h in (256, 512, 1024)}
    c256 = estimate_bpm_tempogram(spec[256], sr, 256, lo, hi, res, band)[3][:aux_k]
    c512 = estimate_bpm_tempogram(spec[512], sr, 512, lo, hi, res, band)[3][:top_k]
    c1024 = estimate_bpm_tempogram(spec[1024], sr, 1024, lo, hi, res, band)[3][:aux_k]
    w512, w256, w1024, dt = mr["w512"], mr["w256"], mr["w1024"], mr["dt512"]

    def lk(c, b):
        return cand_lookup(c, b, tol, ties)

    hyps = []
    for t in [c[0] for c in c512[:top_k]]:
        if not (math.isfinite(t) and t > 0):
            continue
        st = (lk(c512, t), lk(c256, t), lk(c1024, t))
        s2 = (lk(c512, 2 * t), lk(c256, 2 * t), lk(c1024, 2 * t))
        sh = (lk(c512, 0.5 * t), lk(c256, 0.5 * t), lk(c1024, 0.5 * t))
        h_t = w512 * st[0] + w256 * st[1] + w1024 * st[2]
        h_2t = w512 * (dt * st[0] + (1 - dt) * s2[0]) + w256 * s2[1] + w1024 * s2[2]
        h_h = w512 * (dt * st[0] + (1 - dt) * sh[0]) + w256 * sh[1] + w1024 * sh[2]
        if ties.gt("mr-1024-half", st[2], sh[2] * 1.02):
            h_h *= 0.90
        if ties.gt("mr-1024-2t", st[2], s2[2] * 1.02):
            h_2t *= 0.90
        eps = 1e-6
        r2 = (s2[1] + eps) / (st[1] + eps)
        if not ties.ge("mr-r2-110", r2, 1.10):
            h_2t *= 0.75
        if not ties.ge("mr-r2-100", r2, 1.00):
            h_2t *= 0.75
        rh = (sh[2] + eps) / (st[2] + eps)
        if not ties.ge("mr-rh-110", rh, 1.10):
            h_h *= 0.75
        if not ties.ge("mr-rh-100", rh, 1.00):
            h_h *= 0.75
        local = [(b, s) for b, s in ((t, h_t), (2 * t, h_2t), (0.5 * t, h_h)) if lo <= b <= hi]
        local = [(b, s * (0.80 if b > 210.0 else 0.90 if b > 180.0 else 0.92 if b < 60.0 else 1.0)) for b, s in local]
        if not local:
            continue
        # (a near tie in this order never matters: the two near-equal leaders have a margin below
        # margin_threshold, and either order then keeps T with h_t)
        local.sort(key=lambda h: -h[1])  # stable, as the reference's sort_by
        bb, bs = local[0]
        margin = bs - (local[1][1] if len(local) > 1 else 0.0)
        cb, cs = bb, bs
        below = not ties.ge("mr-margin", margin, mr["margin"])
        if abs(cb - t) > 1e-3 and below:
            cb, cs = t, h_t
        if below and mr["human_prior"] and 70.0 <= cb <= 180.0 and margin < 0.05:
            cs += 0.05
        hyps.append((cb, cs))
    if not hyps:
        raise ValueError("Multi-resolution fusion produced no hypotheses")
    order = sorted(range(len(hyps)), key=lambda i: -hyps[i][1])  # stable, as sort_by
    nov = novelty_full(spec[512], band)

    def finish(order, ties):
        """dedup (:531-546), folds (:697-751), triplet family (:764-867), confidence and agreement
        (:869-886) for one order of the hypotheses"""
        uniq = []
        for i in order:
            h = hyps[i]
            if any(abs(u[0] - h[0]) < 0.75 for u in uniq):
                continue
            uniq.append(h)
            if len(uniq) >= 8:
                break
        best = uniq[0]

        def total_support(b):
            s3 = (cand_lookup(c256, b, tol, ties), cand_lookup(c512, b, tol, ties), cand_lookup(c1024, b, tol, ties))
            return sum(s3), sum(v > 0 for v in s3)

        if best[0] >= 170.0:  # fold-down
            half = best[0] * 0.5
            if 70.0 <= half <= 120.0:
                sb, _ = total_support(best[0])
                sh_, ah = total_support(half)
                ratio = sh_ / sb if sb > 0 else 0.0
                if ah >= 3 and sh_ > 0 and sb > 0 and ties.ge("mr-fold-down", ratio, 0.45):
                    best = (half, sh_)
        if best[0] <= 80.0:  # fold-up
            dbl = best[0] * 2.0
            if 70.0 <= dbl <= 180.0:
                sb, _ = total_support(best[0])
                sd, ad = total_support(dbl)
                ratio = sd / sb if sb > 0 else 0.0
                if ad >= 2 and sd > 0 and sb > 0 and ties.ge("mr-fold-up", ratio, 0.55):
                    best = (dbl, sd)
        if 70.0 <= best[0] <= 180.0 and nov.size:  # triplet / compound family
            fams = []
            for f in (f32(1.0), f32(3.0) / f32(2.0), f32(2.0) / f32(3.0), f32(4.0) / f32(3.0), f32(3.0) / f32(4.0)):
                b = float(f32(f32(best[0]) * f))  # f32 BPM products (:786), discrete like the candidates
                if not (math.isfinite(b) and lo <= b <= hi and 70.0 <= b <= 180.0):
                    continue
                sup, ag = total_support(b)
                if ag < 2 or sup <= 0:
                    continue
                fams.append((b, sup, beat_contrast(nov, sr, 512, b, ties)))
            if len(fams) >= 2:
                bsup = max(max(f[1] for f in fams), 1e-6)
                alt = max([f[1] / bsup for f in fams if abs(f[0] - best[0]) > 0.75] + [0.0])
                if ties.ge("mr-family-alt", alt, 0.45):
                    chosen, cscore = fams[0], -1e9
                    for f in fams:
                        sc = f[2] + 0.35 * min(max(f[1] / bsup, 0.0), 1.0)
                        if ties.gt("mr-family-pick", sc, cscore, 1e-4):
                            chosen, cscore = f, sc
                    cur = beat_contrast(nov, sr, 512, best[0], ties)
                    if abs(chosen[0] - best[0]) > 0.75 and ties.ge("mr-family-align", chosen[2], cur + 0.40, 1e-4):
                        best = (chosen[0], chosen[1])
        second = uniq[1][1] if len(uniq) > 1 else 0.0
        conf = min(max(max(best[1] - second, 0.0) / best[1], 0.0), 1.0) if best[1] > 1e-6 else 0.0
        agree = sum(cand_lookup(c, best[0], tol, ties) > 0 for c in (c256, c512, c1024))
        return best[0], conf, int(agree)

    out = finish(order, ties)
    # hypotheses whose scores differ by less than f32 can resolve may sort either way: the order
    # matters only if the other order changes the result (BPM, agreement, confidence beyond 1e-4)
    for k in range(len(order) - 1):
        a, b = hyps[order[k]], hyps[order[k + 1]]
        if _near(a[1], b[1], SCORE_TIE):
            alt = order[:k] + [order[k + 1], order[k]] + order[k + 2:]
            o2 = finish(alt, Ties())
            if abs(o2[0] - out[0]) > 1e-4 or o2[2] != out[2] or abs(o2[1] - out[1]) > 1e-4:
                ties.append(("mr-hyp-order", a, b))
    return out


def accept_multi_resolution(base, mr_est, trap_low, trap_high, ties=None):
    """The acceptance rule of src/lib.rs:511-545: (bpm, conf, agree) tuples -> used_mr."""
    ties = Ties() if ties is None else ties
    bb, bc, ba = base
    mb, mc, ma = mr_est
    rel = max(mb / bb, bb / mb) if bb > 1e-6 else 1.0
    family = abs(rel - 2.0) < 0.05 or abs(rel - 1.5) < 0.05 or abs(rel - 4.0 / 3.0) < 0.05
    forbid = bb <= 180.0 and mb > 180.0
    return (not forbid) and (ties.ge("acc-conf", mc, bc + 0.05)
                             or (ma > ba and ties.ge("acc-agree", mc, bc * 0.90))
                             or ((trap_low or trap_high) and family and ties.ge("acc-family", mc, bc * 0.88)
                                 and (70.0 <= mb <= 180.0 or bb > 180.0)))


# ---- onset detection (a4, a6, a7, a8) ----
ONSET_DEFAULT = dict(percentile=0.80, tol_ms=50, weights=(0.25, 0.25, 0.25, 0.25), energy_db=-20.0)  # config.rs:601-604


def _peaks(flux, thr, ties, tag):
    """Peak picking shared by the three detectors: interior i (1 <= i < n-1) with flux > thr,
    > prev, >= next; the first value with > thr and >= its successor; the last with > thr and >
    its predecessor.  Returns flux indices, sorted, unique."""
    n = flux.size
    scale = max(float(flux.max()), 1e-30) if n else 1.0

    def gt(a, b):
        if ties is not None and _near(a, b, 1e-6 * scale):
            ties.append((tag, a, b))
        return a > b

    def ge(a, b):
        if ties is not None and _near(a, b, 1e-6 * scale):
            ties.append((tag, a, b))
        return a >= b

    out = [i for i in range(1, n - 1) if gt(flux[i], thr) and gt(flux[i], flux[i - 1]) and ge(flux[i], flux[i + 1])]
    if n > 1 and gt(flux[0], thr) and ge(flux[0], flux[1]):
        out.append(0)
    if n > 1 and gt(flux[n - 1], thr) and gt(flux[n - 1], flux[n - 2]):
        out.append(n - 1)
    return sorted(set(out))


def energy_flux_onsets(x, frame, hop, threshold_db=-20.0, ties=None):
    """detect_energy_flux_onsets (energy_flux.rs:67-243) on samples x: onset sample positions."""
    n = x.size
    if n == 0 or frame > n:
        return []
    nf = (n - frame) // hop + 1
    if nf < 2:
        return []
    x = x.astype(np.float64)
    c = np.concatenate([[0.0], np.cumsum(x * x)])
    s = np.arange(nf) * hop
    rms = np.sqrt((c[s + frame] - c[s]) / frame)
    flux = np.maximum(np.diff(rms), 0.0)
    mx = float(flux.max())
    if mx <= EPS:
        return []
    thr = mx * 10.0 ** (threshold_db / 20.0)
    on = [(i + 1) * hop for i in _peaks(flux, thr, ties, "energy-peak") if (i + 1) * hop < n]
    out = []
    for o in on:  # dedup: at least hop / 2 after the last kept onset
        if not out or o >= out[-1] + hop // 2:
            out.append(o)
    return out


def _percentile_threshold(flux, pct):
    srt = np.sort(flux)
    idx = min(int(f32(f32(srt.size) * f32(pct))), srt.size - 1)  # f32 index arithmetic, truncated
    return float(srt[idx])


def spectral_flux_onsets(M, pct, ties=None):
    """detect_spectral_flux_onsets (spectral_flux.rs:69-221): onset frame indices."""
    if M.shape[0] < 2:
        return []
    mx = M.max(axis=1, initial=0.0)
    N = np.where((mx > EPS)[:, None], M / np.where(mx > EPS, mx, 1.0)[:, None], 0.0)
    d = np.maximum(N[1:] - N[:-1], 0.0)
    flux = np.sqrt((d * d).sum(axis=1))
    return [i + 1 for i in _peaks(flux, _percentile_threshold(flux, pct), ties, "spectral-peak")]


def hfc_onsets(M, pct, ties=None):
    """detect_hfc_onsets (hfc.rs:76-214): onset frame indices."""
    if M.shape[0] < 2:
        return []
    h = (M * M * np.arange(M.shape[1], dtype=np.float64)).sum(axis=1)
    flux = np.maximum(np.diff(h), 0.0)
    return [i + 1 for i in _peaks(flux, _percentile_threshold(flux, pct), ties, "hfc-peak")]


def vote_onsets(lists, weights, tol_ms, sr):
    """vote_onsets (consensus.rs:111-287): clusters in arrival order (an onset joins the first
    cluster holding a member within the tolerance), centre = integer mean, confidence = weight
    share; candidates sorted by confidence, descending, stable."""
    tol = int(f32(f32(f32(tol_ms) / f32(1000.0)) * f32(sr)))  # discrete: the reference's f32 arithmetic
    allo = sorted(((s, m) for m, l in enumerate(lists) for s in l), key=lambda o: o[0])  # stable by sample
    clusters = []
    for s, m in allo:
        for cl in clusters:
            if any(abs(s - e) <= tol for e, _ in cl):
                cl.append((s, m))
                break
        else:
            clusters.append([(s, m)])
    wmax = float(sum(weights))
    cands = []
    for cl in clusters:
        centre = sum(s for s, _ in cl) // len(cl)
        tw = sum(weights[m] for _, m in cl)
        cands.append((centre, min(max(tw / wmax, 0.0), 1.0) if wmax > 0 else 0.0, len({m for _, m in cl})))
    cands.sort(key=lambda c: -c[1])
    return cands


def consensus_onsets(x, sr, M, frame=2048, hop=512, cfg=ONSET_DEFAULT, ties=None):
    """The onset stage of src/lib.rs:152-289 (default config: energy flux on the trimmed samples,
    spectral flux and HFC on the hop spectrogram, consensus vote, >= 2 methods else all).
    Returns (energy, spectral, hfc, chosen) as sample positions."""
    n = x.size
    energy = energy_flux_onsets(x, frame, hop, cfg["energy_db"], ties)

    def to_samples(frames):
        return sorted({f * hop for f in frames if f * hop < n})

    spectral = to_samples(spectral_flux_onsets(M, cfg["percentile"], ties))
    hfc = to_samples(hfc_onsets(M, cfg["percentile"], ties))
    chosen = energy
    if M.shape[0] > 0:
        cands = vote_onsets([energy, spectral, hfc, []], cfg["weights"], cfg["tol_ms"], sr)
        strong = sorted({c[0] for c in cands if c[2] >= 2})
        anyc = sorted({c[0] for c in cands})
        pick = strong if strong else anyc
        if pick:
            chosen = pick
    return energy, spectral, hfc, chosen


# ---- key path (src/lib.rs:961-1540, default AnalysisConfig, config.rs:669-739) ----
# The 8192 / 512 key STFT, the harmonic time mask (extractor.rs:1246-1349, margin 12, power 2),
# HPCP (extractor.rs:529-680, 1097-1150: peaks 24, harmonics 4, decay 0.6, magnitude power 0.5,
# sigma 0.5, 100-5000 Hz, no tuning or whitening), the 5-frame median (smoothing.rs:37-94), the
# frame weights (lib.rs:1236-1287: tonalness^2 x (energy / median)^0.5), segment voting
# (lib.rs:1331-1436: 1024-frame segments, hop 512, clarity >= 0.2) over detect_key_weighted
# (detector.rs:68-313, Krumhansl-Kessler templates, templates.rs:64-140) and the key clarity
# (key_clarity.rs:51-93).  Float64 throughout.
KK_MAJOR = (6.35, 2.23, 3.48, 2.33, 4.38, 4.09, 2.52, 5.19, 2.39, 3.66, 2.29, 2.88)
KK_MINOR = (6.33, 2.68, 3.52, 5.38, 2.60, 3.53, 2.54, 4.75, 3.98, 2.69, 3.34, 3.17)
KEY_DEFAULT = dict(margin=12, mask_power=2.0, peaks=24, harmonics=4, decay=0.6, mag_power=0.5, sigma=0.5,
                   fmin=100.0, fmax=5000.0, tonal_pow=2.0, energy_pow=0.5, min_tonal=0.0, seg_len=1024, seg_hop=512,
                   min_clarity=0.2)


def key_templates64():
    """(major[12][12], minor[12][12]): the base profiles rotated to every tonic, L2-normalised."""
    def rot(base):
        t = np.array([[base[(s + 12 - k) % 12] for s in range(12)] for k in range(12)], np.float64)
        n = np.sqrt((t * t).sum(axis=1))
        return t / np.where(n > 1e-12, n, 1.0)[:, None]
    return rot(KK_MAJOR), rot(KK_MINOR)


def harmonic_mask64(M, margin=12, power=2.0):
    """harmonic_spectrogram_time_mask: X * H^p / (H^p + max(X - H, 0)^p + 1e-12), H the moving
    average over frames t - margin .. t + margin (clipped to the track)."""
    M = np.asarray(M, np.float64)
    F = M.shape[0]
    if F == 0:
        return M
    P = np.vstack([np.zeros((1, M.shape[1])), np.cumsum(M, axis=0)])
    t = np.arange(F)
    st, en = np.maximum(t - margin, 0), np.minimum(t + margin + 1, F)
    H = (P[en] - P[st]) / np.maximum(en - st, 1)[:, None]
    p = max(power, 1.0)
    x, h = np.maximum(M, 0.0), np.maximum(H, 0.0)
    r = np.maximum(x - h, 0.0)
    hp, rp = h ** p, r ** p
    return x * (hp / (hp + rp + 1e-12))


def hpcp64(M, sr, fft_size, cfg=KEY_DEFAULT):
    """Per-frame HPCP (frame_to_hpcp_tuned_band) and frame energies sum(x^2).  The top-K peaks are
    taken by magnitude, ties broken by the lower bin (the reference's select_nth_unstable order is
    unspecified; the sum is order-insensitive but for rounding)."""
    M = np.asarray(M, np.float64)
    F, nb = M.shape
    energy = (M * M).sum(axis=1)
    pc = np.zeros((F, 12))
    fres = sr / fft_size
    fmin, fmax = max(cfg["fmin"], 20.0), min(cfg["fmax"], sr / 2.0)
    b = np.arange(1, nb - 1)
    fb = b * fres
    b = b[(fb >= fmin) & (fb <= fmax)]
    if F == 0 or b.size == 0:
        return pc, energy
    m, mp, mn = M[:, b], M[:, b - 1], M[:, b + 1]
    cand = ~((m <= mp) | (m < mn))
    score = np.where(cand, m, -np.inf)
    k = cfg["peaks"]
    # stable descending order by magnitude, the lower bin first among equals
    order = np.argsort(-score, axis=1, kind="stable")[:, :k]
    sigma, decay, p = max(cfg["sigma"], 1e-6), min(max(cfg["decay"], 0.0), 1.0), min(max(cfg["mag_power"], 0.05), 1.0)
    rows = np.arange(F)[:, None]
    ok = np.isfinite(score[rows, order])
    pbin = b[order]
    w0 = np.where(ok, np.maximum(M[rows, pbin], 0.0) ** p, 0.0)
    f0 = pbin * fres
    for h in range(1, max(cfg["harmonics"], 1) + 1):
        fh = f0 * h
        live = ok & (w0 > 0) & (f0 > 0) & (fh >= fmin) & (fh <= fmax)
        # a harmonic above fmax ends the peak's loop; below fmin only skips it (h grows)
        semi = 12.0 * np.log2(np.where(live, fh, 440.0) / 440.0) + 57.0
        spc = np.mod(semi, 12.0)
        prim = np.mod(np.floor(spc + 0.5), 12.0).astype(int)  # f32::round (half away; spc >= 0)
        hw = decay ** (h - 1) / h
        for off in (-1, 0, 1):
            tc = (prim + off) % 12
            d = np.abs(spc - tc)
            d = np.minimum(d, 12.0 - d)
            wgt = np.exp(-d * d / (2.0 * sigma * sigma))
            np.add.at(pc, (np.broadcast_to(rows, tc.shape)[live], tc[live]), (w0 * hw * wgt)[live])
    n = np.sqrt((pc * pc).sum(axis=1))
    pc = np.where((n > 1e-10)[:, None], pc / np.where(n > 1e-10, n, 1.0)[:, None], pc)
    return pc, energy


def smooth_chroma64(C, window=5):
    """smooth_chroma: per pitch class, the median of the frames t - 2 .. t + 2 present in the
    track (element len // 2 of the sorted window)."""
    C = np.asarray(C, np.float64)
    F = C.shape[0]
    half = window // 2
    out = np.empty_like(C)
    for t in range(F):
        w = np.sort(C[max(t - half, 0):min(t + half + 1, F)], axis=0)
        out[t] = w[w.shape[0] // 2]
    return out


def key_weights64(C, E, cfg=KEY_DEFAULT):
    """The frame weights of lib.rs:1236-1287, or None where the reference falls back to unweighted."""
    s = C.sum(axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        P = C / np.where(s > 1e-12, s, 1.0)[:, None]
        ent = -np.where(P > 1e-12, P * np.log(np.where(P > 1e-12, P, 1.0)), 0.0).sum(axis=1)
    tonal = np.where(s <= 1e-12, 0.0, np.clip(1.0 - ent / math.log(12.0), 0.0, 1.0))
    tonal = np.where(tonal < cfg["min_tonal"], 0.0, tonal)
    med = max(float(np.sort(E)[E.size // 2]), 1e-12)
    w = np.maximum(tonal ** max(cfg["tonal_pow"], 0.0) * np.maximum(E / med, 0.0) ** max(cfg["energy_pow"], 0.0), 0.0)
    if w.sum() <= 1e-12 or int((w > 0).sum()) < 10:
        return None
    return w


def key_clarity64(scores):
    """compute_key_clarity over (key, score) pairs in the caller's order: (first - mean) / range."""
    v = np.array([s for _, s in scores], np.float64)
    if v.size < 2:
        return 0.0
    rng = v.max() - v.min()
    return float(np.clip((v[0] - v.mean()) / rng, 0.0, 1.0)) if rng > 1e-10 else 0.0


def detect_key_weighted64(C, w, templates):
    """detect_key_weighted: (sorted (key, score) list, key, confidence); key k < 12 major, else
    minor k - 12.  The top-3 HashMap vote's pick is unspecified in the reference (iteration
    order); like the CPU restatement this takes the first sorted key."""
    maj, mnr = templates
    ww = np.ones(C.shape[0]) if w is None else np.where(w > 0, w, 0.0)
    raw = np.concatenate([(C @ maj.T * ww[:, None]).sum(axis=0), (C @ mnr.T * ww[:, None]).sum(axis=0)])
    mM, mm = max(0.0, raw[:12].max()), max(0.0, raw[12:].max())
    sc = raw.copy()
    if mM > 1e-9 and mm > 1e-9:
        sc[:12] /= mM
        sc[12:] /= mm
    tM = 11 - int(np.argmax(sc[:12][::-1]))  # max_by keeps the last maximum
    tm = 11 - int(np.argmax(sc[12:][::-1]))
    cof = [0, 7, 2, 9, 4, 11, 6, 1, 8, 3, 10, 5]
    ref = sc.copy()
    for k in range(24):
        rt, rs = (tM, sc[tM]) if k < 12 else (tm, sc[12 + tm])
        if rs > 1e-9:
            d = abs(cof.index(k % 12) - cof.index(rt))
            d = min(d, 12 - d)
            if d <= 2:
                ref[k] += rs * (0.20 * (1.0 - d * 0.5))
    order = sorted(range(24), key=lambda k: -ref[k])  # stable: majors, then minors, by index
    scores = [(k, float(ref[k])) for k in order]
    best = scores[0][1]
    conf = float(np.clip((best - scores[1][1]) / best, 0.0, 1.0)) if best > 0 else 0.0
    return scores, scores[0][0], conf


def key_path64(M8, sr, fft_size=8192, cfg=KEY_DEFAULT, ties=None):
    """(key, confidence, clarity) of the default key path from an 8192-point magnitude spectrogram
    (frames x bins); ties (ref64.Ties) records segments whose clarity is within 1e-4 of the
    threshold, where the reference's f32 rounding decides whether the segment votes."""
    H = harmonic_mask64(M8, cfg["margin"], cfg["mask_power"])
    C, E = hpcp64(H, sr, fft_size, cfg)
    if C.shape[0] > 5:
        C = smooth_chroma64(C, 5)
    w = key_weights64(C, E, cfg)
    T = key_templates64()
    F = C.shape[0]
    if F >= max(cfg["seg_len"], 1) and cfg["seg_len"] >= 120:
        L = min(cfg["seg_len"], F)
        hop = max(min(cfg["seg_hop"], L), 1)
        acc = np.zeros(24)
        used = 0
        for st in range(0, F - L + 1, hop):
            scores, _, _ = detect_key_weighted64(C[st:st + L], None if w is None else w[st:st + L], T)
            cl = key_clarity64(scores)
            if ties is not None and abs(cl - cfg["min_clarity"]) < 1e-4:
                ties.append(("segment-clarity", cl, cfg["min_clarity"]))
            if cl >= cfg["min_clarity"]:
                used += 1
                for k, s in scores:
                    acc[k] += s * cl
        if used:
            order = sorted(range(24), key=lambda k: -acc[k])
            scores = [(k, float(acc[k])) for k in order]
            best = scores[0][1]
            conf = float(np.clip((best - scores[1][1]) / best, 0.0, 1.0)) if best > 0 else 0.0
            return scores[0][0], conf, key_clarity64(scores)
    scores, key, conf = detect_key_weighted64(C, w, T)
    return key, conf, key_clarity64(scores)
