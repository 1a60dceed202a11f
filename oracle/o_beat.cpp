// o_beat.cpp — beat grid (TEST INFRASTRUCTURE, see oracle_internal.hpp).
//
// Follows src/features/beat_tracking/{mod.rs:108-485, hmm.rs:121-441, tempo_variation.rs:95-227,
// bayesian.rs:77-272, time_signature.rs:90-199}.
#include <algorithm>
#include <array>

#include "oracle_internal.hpp"

namespace orc {

struct BeatPos {
    float t, conf;
};

// hmm.rs:165-174: tempo states 0.90 .. 1.10 x the estimate
static void hmm_states(float bpm, float out[5]) {
    const float mult[5] = {0.90f, 0.95f, 1.00f, 1.05f, 1.10f};
    for (int i = 0; i < 5; i++) out[i] = bpm * mult[i];
}

// hmm.rs:184-219: transition matrix, rows normalized
static void hmm_transition(float T[5][5]) {
    for (int i = 0; i < 5; i++) {
        float sum = 0.0f;
        for (int j = 0; j < 5; j++) {
            const int d = i > j ? i - j : j - i;
            T[i][j] = d == 0 ? 0.7f : d == 1 ? 0.15f : 0.0f;
            sum += T[i][j];
        }
        if (sum > EPS)
            for (int j = 0; j < 5; j++) T[i][j] /= sum;
    }
}

// hmm.rs:121-441.  The Viterbi pass is run faithfully, but note that the
// emission is state-independent, so the extracted beats never depend on the path.
static bool hmm_track(float bpm, const std::vector<float>& on, std::vector<BeatPos>* out) {
    if (bpm <= EPS || bpm > 300.0f) return false;  // InvalidInput
    if (on.empty()) return false;
    const float start = on[0], end = on.back();
    const float interval = 60.0f / bpm;
    const size_t nf = (size_t)sd_f2u64(__builtin_ceilf((end - start) / interval)) + 1;
    const float sigma = 0.05f / 2.0f;
    const float sigma_sq = sigma * sigma;
    std::vector<float> emis(nf);
    for (size_t t = 0; t < nf; t++) {
        const float ft = start + ((float)t * interval);
        float md = SD_INF_F;
        for (float o : on) {
            const float d = sd_absf(o - ft);
            if (d < md) md = d;
        }
        const float dsq = md * md;
        emis[t] = sd_expf(-dsq / (2.0f * sigma_sq));  // identical for all 5 states
    }
    float T[5][5];
    hmm_transition(T);
    // Viterbi (hmm.rs:308-375)
    std::vector<float> v(5), nv(5);
    std::vector<std::array<int, 5>> bp(nf);
    for (int s = 0; s < 5; s++) v[s] = (1.0f / 5.0f) * emis[0];
    for (size_t t = 1; t < nf; t++) {
        for (int s = 0; s < 5; s++) {
            float best = 0.0f;
            int bs = 0;
            for (int ps = 0; ps < 5; ps++) {
                const float p = v[ps] * T[ps][s];
                if (p > best) {
                    best = p;
                    bs = ps;
                }
            }
            nv[s] = best * emis[t];
            bp[t][s] = bs;
        }
        v.swap(nv);
    }
    // (path irrelevant to the output; extract beats, hmm.rs:383-441)
    out->clear();
    for (size_t t = 0; t < nf; t++) {
        const float e = emis[t];
        if (e > 0.1f) {
            const float bt = start + ((float)t * interval);
            float md = SD_INF_F;
            for (float o : on) {
                const float d = sd_absf(o - bt);
                if (d < md) md = d;
            }
            const float align = md < 0.05f ? 1.0f - (md / 0.05f) : 0.0f;
            out->push_back({bt, sd_minf(e * 0.7f + align * 0.3f, 1.0f)});
        }
    }
    std::stable_sort(out->begin(), out->end(), [](auto& a, auto& b) { return a.t < b.t; });
    return true;
}

struct Seg {
    float start, end, bpm, conf;
    bool variable;
};

// tempo_variation.rs:95-227
static std::vector<Seg> tempo_variations(const std::vector<float>& b, float nominal) {
    if (b.size() < 4) return {{b.empty() ? 0.0f : b[0], b.empty() ? 0.0f : b.back(), nominal, 0.5f, false}};
    if (nominal <= EPS) fail(SDSP_ERR_INVALID_INPUT, "Invalid nominal BPM");
    const float total = b.back() - b[0];
    if (total < 2.0f) return {{b[0], b.back(), nominal, 0.8f, false}};
    const float seg_dur = sd_clampf(total / 4.0f, 4.0f, 8.0f);
    const float overlap = seg_dur * 0.5f;
    std::vector<Seg> segs;
    float cur = b[0];
    while (cur < b.back()) {
        const float se = sd_minf(cur + seg_dur, b.back());
        std::vector<float> sb;
        for (float x : b)
            if (x >= cur && x <= se) sb.push_back(x);
        if (sb.size() >= 3) {
            std::vector<float> iv;
            for (size_t i = 1; i < sb.size(); i++) {
                const float d = sb[i] - sb[i - 1];
                if (d > 0.0f) iv.push_back(d);
            }
            if (!iv.empty()) {
                float sum = 0.0f;
                for (float x : iv) sum += x;
                const float mean = sum / (float)iv.size();
                float vs = 0.0f;
                for (float x : iv) {
                    const float d = x - mean;
                    vs += d * d;
                }
                const float var = vs / (float)iv.size();
                const float sd = __builtin_sqrtf(var);
                const float cv = mean > EPS ? sd / mean : 0.0f;
                const float sbpm = mean > EPS ? 60.0f / mean : nominal;
                const float conf = sd_maxf(1.0f - sd_minf(cv / 0.3f, 1.0f), 0.0f);
                segs.push_back({cur, se, sbpm, conf, cv > 0.15f});
            }
        }
        cur += seg_dur - overlap;
    }
    if (segs.empty()) segs.push_back({b[0], b.back(), nominal, 0.8f, false});
    return segs;
}

// bayesian.rs:104-272 (tracker state carried across segments)
struct Bayes {
    float bpm, conf;
    std::vector<float> history;  // BayesianBeatTracker::history (new(): [initial])
};
static Bayes bayes_new(float bpm, float conf) { return {bpm, sd_clampf(conf, 0.0f, 1.0f), {bpm}}; }  // :77-83
// generate_bpm_candidates (:183-199): f32 0.5-BPM steps over [max(bpm-5, 60), min(bpm+5, 180)]
static std::vector<float> bayes_candidates(const Bayes& st) {
    std::vector<float> c;
    const float lo = sd_maxf(st.bpm - 5.0f, 60.0f), hi = sd_minf(st.bpm + 5.0f, 180.0f);
    for (float b = lo; b <= hi; b += 0.5f) c.push_back(b);
    return c;
}
// compute_likelihood (:201-252): exp of the mean Gaussian log-likelihood (sigma 0.05 s) of the
// onsets' distances to the nearest grid beat anchored at the first onset
static float bayes_likelihood(const std::vector<float>& on, float cb) {
    if (cb <= EPS) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM for likelihood");
    if (on.empty()) return 0.0f;
    const float bi = 60.0f / cb;
    const float st0 = on[0];
    float ll = 0.0f;
    int32_t valid = 0;
    const float sig_sq = 0.05f * 0.05f;
    for (float o : on) {
        const int32_t idx = sd_f2i32(sd_roundf((o - st0) / bi));
        const float exp_t = st0 + ((float)idx * bi);
        const float d = sd_absf(o - exp_t);
        const float dsq = d * d;
        ll += -dsq / (2.0f * sig_sq);
        valid++;
    }
    return valid == 0 ? 0.0f : sd_expf(ll / (float)valid);
}
// compute_prior (:254-265): Gaussian in the BPM change, sigma 2 BPM
static float bayes_prior(const Bayes& st, float bpm) {
    const float d = sd_absf(bpm - st.bpm);
    const float sig_sq = 2.0f * 2.0f;
    return sd_expf(-(d * d) / (2.0f * sig_sq));
}
static void bayes_update(Bayes& st, const std::vector<float>& on, float* out_bpm) {
    if (on.empty()) fail(SDSP_ERR_INVALID_INPUT, "Cannot update: no onsets provided");
    if (st.bpm <= EPS || st.bpm > 300.0f) fail(SDSP_ERR_INVALID_INPUT, "Invalid current BPM");
    float best_bpm = st.bpm, best_l = 0.0f;
    for (float cb : bayes_candidates(st)) {
        const float lik = bayes_likelihood(on, cb);
        if (lik > best_l) {
            best_l = lik;
            best_bpm = cb;
        }
    }
    (void)bayes_prior(st, best_bpm);  // the posterior (:140-141) is computed and unused
    const float old = st.bpm;
    st.bpm = best_bpm;
    st.history.push_back(best_bpm);
    const float ch = sd_absf(best_bpm - old);
    const float pen = ch < 1.0f ? 1.0f : ch < 3.0f ? 0.8f : 0.5f;
    st.conf = sd_minf(best_l * pen, 1.0f);
    *out_bpm = st.bpm;
}

// time_signature.rs:161-199
static float score_ts(const std::vector<float>& iv, uint32_t bpb, float mean) {
    if (iv.size() < bpb) return 0.0f;
    const size_t lag = bpb;
    float acc = 0.0f;
    int32_t cnt = 0;
    for (size_t i = 0; i + lag < iv.size(); i++) {
        const float d = sd_absf(iv[i] - iv[i + lag]);
        acc += 1.0f / (1.0f + d / mean);
        cnt++;
    }
    if (cnt == 0) return 0.0f;
    const float ac = acc / (float)cnt;
    float vs = 0.0f;
    for (float x : iv) {
        const float d = x - mean;
        vs += d * d;
    }
    const float var = vs / (float)iv.size();
    const float cv = mean > EPS ? __builtin_sqrtf(var) / mean : 1.0f;
    const float cons = 1.0f / (1.0f + cv);
    return sd_minf(ac * 0.7f + cons * 0.3f, 1.0f);
}

// time_signature.rs:90-149 -> beats per bar (+ confidence = the best score clamped to [0, 1])
static uint32_t time_signature(const std::vector<float>& b, float bpm, float* conf = nullptr) {
    float dummy;
    if (!conf) conf = &dummy;
    *conf = 0.5f;
    if (b.size() < 8) return 4;
    if (bpm <= EPS) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM for time signature detection");
    std::vector<float> iv;
    for (size_t i = 1; i < b.size(); i++) {
        const float d = b[i] - b[i - 1];
        if (d > 0.0f) iv.push_back(d);
    }
    if (iv.empty()) return 4;
    float sum = 0.0f;
    for (float x : iv) sum += x;
    const float mean = sum / (float)iv.size();
    const float s44 = score_ts(iv, 4, mean), s34 = score_ts(iv, 3, mean), s68 = score_ts(iv, 6, mean);
    // max_by with partial_cmp: the LAST maximum wins
    uint32_t best = 4;
    float bs = s44;
    if (!(s34 < bs)) {
        best = 3;
        bs = s34;
    }
    if (!(s68 < bs)) {
        best = 6;
        bs = s68;
    }
    *conf = sd_clampf(bs, 0.0f, 1.0f);
    return best;
}

// beat_tracking/mod.rs:108-247 (+ downbeats :363-404, stability :425-485)
bool generate_beat_grid(float bpm, float conf, const std::vector<float>& onsets_s, uint32_t sr,
                        std::vector<float>* beats_out, std::vector<float>* down_out, float* stab_out,
                        BeatDiag* diag) {
    (void)sr;
    BeatDiag dg;
    try {
        if (bpm <= 0.0f || bpm > 300.0f) return false;
        if (onsets_s.empty()) return false;
        std::vector<float> on(onsets_s);
        std::stable_sort(on.begin(), on.end(), [](float a, float b) { return a < b; });
        std::vector<BeatPos> pos;
        if (!hmm_track(bpm, on, &pos)) return false;
        if (pos.empty()) return false;  // ProcessingError
        std::vector<float> bt;
        for (auto& p : pos) bt.push_back(p.t);
        auto segs = tempo_variations(bt, bpm);
        bool var = false;
        for (auto& s : segs) var |= s.variable;
        dg.variable = var;
        if (var) {
            std::vector<BeatPos> refined;
            Bayes st = bayes_new(bpm, conf);
            for (auto& s : segs) {
                if (s.variable) {
                    std::vector<float> so;
                    for (float o : on)
                        if (o >= s.start && o <= s.end) so.push_back(o);
                    if (!so.empty()) {
                        float ub;
                        bayes_update(st, so, &ub);
                        std::vector<BeatPos> sb;
                        if (hmm_track(ub, so, &sb)) refined.insert(refined.end(), sb.begin(), sb.end());
                    }
                } else {
                    for (auto& p : pos)
                        if (p.t >= s.start && p.t <= s.end) refined.push_back(p);
                }
            }
            if (!refined.empty()) {
                std::stable_sort(refined.begin(), refined.end(), [](auto& a, auto& b) { return a.t < b.t; });
                pos.swap(refined);
                dg.refined = true;
            }
        }
        bt.clear();
        for (auto& p : pos) bt.push_back(p.t);
        const uint32_t bpb = time_signature(bt, bpm);
        dg.beats_per_bar = bpb;
        // generate_beat_grid_from_positions_with_time_sig (:290-320)
        std::vector<float> beats(bt);
        std::stable_sort(beats.begin(), beats.end(), [](float a, float b) { return a < b; });
        std::vector<float> down;
        if (!beats.empty()) {
            const float bi = 60.0f / bpm;
            const float bar = bi * (float)bpb;
            const float tol = bar * 0.1f;
            down.push_back(beats[0]);
            for (size_t i = 1; i < beats.size(); i++) {
                const float exp_t = down.back() + bar;
                if (sd_absf(beats[i] - exp_t) <= tol) down.push_back(beats[i]);
            }
        }
        // calculate_grid_stability
        float stab = 0.0f;
        if (pos.size() >= 2) {
            std::vector<float> iv;
            for (size_t i = 1; i < pos.size(); i++) {
                const float d = pos[i].t - pos[i - 1].t;
                if (d > 0.0f) iv.push_back(d);
            }
            if (!iv.empty()) {
                float sum = 0.0f;
                for (float x : iv) sum += x;
                const float mean = sum / (float)iv.size();
                if (mean > 1e-10f) {
                    float vs = 0.0f;
                    for (float x : iv) {
                        const float d = x - mean;
                        vs += d * d;
                    }
                    const float var = vs / (float)iv.size();
                    const float cv = __builtin_sqrtf(var) / mean;
                    stab = 1.0f / (1.0f + cv);
                }
            }
        }
        *beats_out = beats;
        *down_out = down;
        *stab_out = stab;
        if (diag) *diag = dg;
        return true;
    } catch (const AErr&) {
        return false;  // src/lib.rs:932-943: any error -> empty grid, stability 0
    }
}

}  // namespace orc

// ---- KAT probes (tests only) ----
extern "C" void sdsp_oracle_hmm_model(float bpm, float* states5, float* trans25) {
    orc::hmm_states(bpm, states5);
    float T[5][5];
    orc::hmm_transition(T);
    for (int i = 0; i < 25; i++) trans25[i] = T[i / 5][i % 5];
}

// HmmBeatTracker::track_beats on onset times (s); returns the beat count or -1 (Err)
extern "C" int32_t sdsp_oracle_hmm_track(float bpm, const float* on, int32_t n, float* out, int32_t cap) {
    std::vector<float> v(on, on + (n > 0 ? n : 0));
    std::vector<orc::BeatPos> pos;
    if (!orc::hmm_track(bpm, v, &pos)) return -1;
    const int32_t m = (int32_t)pos.size();
    for (int32_t i = 0; i < m && i < cap; i++) out[i] = pos[(size_t)i].t;
    return m;
}


// ---- unit probes (tests only; tests/test_oracle_units_beat.py) ----
using namespace orc;

extern "C" {

// generate_beat_grid (mod.rs:108-247): the reference returns Err for bpm <= 0 or > 300, empty
// onsets and a failed HMM; the oracle maps every such case to "no grid" (-1 here).
// counts = (beats, downbeats); bars == downbeats (mod.rs:316)
int32_t sdsp_oracle_beat_grid(float bpm, float conf, const float* on, uint64_t n, uint32_t sr, float* beats,
                              float* downs, uint64_t cap, uint64_t* counts, float* stability) {
    std::vector<float> o(on, on + n), b, d;
    float st = 0.0f;
    if (!generate_beat_grid(bpm, conf, o, sr, &b, &d, &st)) return -1;
    for (size_t i = 0; i < b.size() && i < cap; i++) beats[i] = b[i];
    for (size_t i = 0; i < d.size() && i < cap; i++) downs[i] = d[i];
    counts[0] = b.size();
    counts[1] = d.size();
    *stability = st;
    return 0;
}

// detect_downbeats_with_time_sig (mod.rs:363-404)
int64_t sdsp_oracle_downbeats(const float* beats, uint64_t n, float bpm, uint32_t beats_per_bar, float* out) {
    return probe_call([&]() -> int64_t {
        if (n == 0) return 0;
        if (bpm <= 0.0f) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM for downbeat detection");
        const float bar = (60.0f / bpm) * (float)beats_per_bar;
        const float tol = bar * 0.1f;
        int64_t k = 0;
        out[k++] = beats[0];
        for (uint64_t i = 1; i < n; i++)
            if (sd_absf(beats[i] - (out[k - 1] + bar)) <= tol) out[k++] = beats[i];
        return k;
    });
}

// calculate_grid_stability (mod.rs:425-485) over beat times
int32_t sdsp_oracle_grid_stability(const float* t, uint64_t n, float bpm, float* out) {
    return (int32_t)probe_call([&]() -> int64_t {
        *out = 0.0f;
        if (n < 2) return 0;
        if (bpm <= 0.0f) fail(SDSP_ERR_INVALID_INPUT, "Invalid BPM for stability calculation");
        std::vector<float> iv;
        for (uint64_t i = 1; i < n; i++)
            if (t[i] - t[i - 1] > 0.0f) iv.push_back(t[i] - t[i - 1]);
        if (iv.empty()) return 0;
        float sum = 0.0f;
        for (float x : iv) sum += x;
        const float mean = sum / (float)iv.size();
        if (mean <= 1e-10f) return 0;
        float vs = 0.0f;
        for (float x : iv) vs += (x - mean) * (x - mean);
        *out = 1.0f / (1.0f + __builtin_sqrtf(vs / (float)iv.size()) / mean);
        return 0;
    });
}

// detect_tempo_variations (tempo_variation.rs:95-227): 5 floats per segment
// (start, end, bpm, confidence, is_variable); returns the segment count
int64_t sdsp_oracle_tempo_variations(const float* beats, uint64_t n, float nominal, float* out, uint64_t cap) {
    return probe_call([&]() -> int64_t {
        const auto segs = tempo_variations(std::vector<float>(beats, beats + n), nominal);
        for (size_t i = 0; i < segs.size() && i < cap; i++) {
            const float v[5] = {segs[i].start, segs[i].end, segs[i].bpm, segs[i].conf, segs[i].variable ? 1.0f : 0.0f};
            std::memcpy(out + 5 * i, v, sizeof v);
        }
        return (int64_t)segs.size();
    });
}

// BayesianBeatTracker (bayesian.rs:77-272) created with (bpm, conf):
//   op 0: generate_bpm_candidates -> out (returns the count)
//   op 1: compute_likelihood(onsets, x) -> out[0]
//   op 2: compute_prior(x) -> out[0]
//   op 3: new() state -> out = (current_bpm, current_confidence, history...)
//   op 4: update_with_onsets(onsets) -> out = (current_bpm, current_confidence, history...)
// ops 3-4 return the history length
int64_t sdsp_oracle_bayes(int32_t op, float bpm, float conf, const float* on, uint64_t n, float x, float* out,
                          uint64_t cap) {
    return probe_call([&]() -> int64_t {
        Bayes st = bayes_new(bpm, conf);
        const std::vector<float> o(on, on + n);
        switch (op) {
            case 0: {
                const auto c = bayes_candidates(st);
                for (size_t i = 0; i < c.size() && i < cap; i++) out[i] = c[i];
                return (int64_t)c.size();
            }
            case 1: out[0] = bayes_likelihood(o, x); return 0;
            case 2: out[0] = bayes_prior(st, x); return 0;
            default: break;
        }
        if (op == 4) {
            float ub;
            bayes_update(st, o, &ub);
        }
        out[0] = st.bpm;
        out[1] = st.conf;
        for (size_t i = 0; i < st.history.size() && i + 2 < cap; i++) out[2 + i] = st.history[i];
        return (int64_t)st.history.size();
    });
}

// detect_time_signature (time_signature.rs:90-149): beats per bar (4 / 3 / 6) and confidence
int32_t sdsp_oracle_time_signature(const float* beats, uint64_t n, float bpm, uint32_t* bpb, float* conf) {
    return (int32_t)probe_call([&]() -> int64_t {
        *bpb = time_signature(std::vector<float>(beats, beats + n), bpm, conf);
        return 0;
    });
}
}
