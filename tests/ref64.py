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
    bpm = np.arange(P // 2 + 1) * ((sr / hop) / P) * 60.0
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
    cands = sorted(x for b in seed_bpms for f in (1.0, 0.5, 2.0, 1 / 3, 3.0, 2 / 3, 1.5)
                   for x in [b * f] if np.isfinite(x) and lo <= x <= hi)
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
