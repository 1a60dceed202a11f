"""Parity of the opt-in key chroma front-ends against the oracle.

Each case switches the key path's spectrogram conditioning or chroma front-end
(src/lib.rs:1011-1198): the HPSS median mask (extractor.rs:1369-1501), time smoothing without the
mask, no conditioning, plain
frame_to_chroma (soft / hard), tuning compensation (extractor.rs:66-177) with HPCP and with plain
chroma, HPCP whitening and bass blend (extractor.rs:529-680, 1154-1244), the log-frequency
spectrogram (extractor.rs:701-985) and beat-synchronous chroma (extractor.rs:830-935).  A ragged
batch (one track pitch-shifted by +0.3 semitone so that the tuning estimate is non-trivial) runs
through the C ABI and every result field is compared with the oracle (oracle/o_chroma.cpp) on the
same inputs: key exact, floats bit-exact.  The reference holds no golden vectors for these
branches; see tests/test_oracle_chroma.py for how the restatement is pinned.
"""
import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu

SR = 44100


def _tracks():
    out = [synth.make_track(s, seconds=sec, mode=m)[0] for s, sec, m in ((3, 30.0, 1), (11, 24.0, 0), (29, 12.0, None))]
    # rendered at sr * 2^(-0.3/12), analysed at sr: every partial sits 0.3 semitone sharp
    out.append(synth.make_track(53, seconds=40.0, sr=int(round(SR * 2 ** (-0.3 / 12))), mode=0)[0])
    return out


_TRACKS = None


def tracks():
    global _TRACKS
    if _TRACKS is None:
        _TRACKS = _tracks()
    return _TRACKS


CASES = {
    "time_smooth": dict(enable_key_harmonic_mask=0, enable_key_spectrogram_time_smoothing=1),
    "time_smooth_m3": dict(enable_key_harmonic_mask=0, enable_key_spectrogram_time_smoothing=1,
                           key_spectrogram_smooth_margin=3),
    "raw_spectrogram": dict(enable_key_harmonic_mask=0, enable_key_spectrogram_time_smoothing=0),
    "plain_soft": dict(enable_key_hpcp=0),
    "plain_hard": dict(enable_key_hpcp=0, soft_chroma_mapping=0),
    "plain_sigma": dict(enable_key_hpcp=0, soft_mapping_sigma=0.9),
    "tuning_hpcp": dict(enable_key_tuning_compensation=1),
    "tuning_hpcp_wide": dict(enable_key_tuning_compensation=1, key_tuning_max_abs_semitones=0.5,
                             key_tuning_frame_step=7, key_tuning_peak_rel_threshold=0.2),
    "tuning_plain": dict(enable_key_hpcp=0, enable_key_tuning_compensation=1, key_tuning_max_abs_semitones=0.5),
    "tuning_plain_hard": dict(enable_key_hpcp=0, soft_chroma_mapping=0, enable_key_tuning_compensation=1,
                              key_tuning_max_abs_semitones=0.5),
    "whitening": dict(enable_key_hpcp_whitening=1),
    "whitening_7": dict(enable_key_hpcp_whitening=1, key_hpcp_whitening_smooth_bins=7),
    "whitening_off_small": dict(enable_key_hpcp_whitening=1, key_hpcp_whitening_smooth_bins=2),
    "bass_blend": dict(enable_key_hpcp_bass_blend=1),
    "bass_white_tuned": dict(enable_key_hpcp_bass_blend=1, enable_key_hpcp_whitening=1,
                             enable_key_tuning_compensation=1, key_tuning_max_abs_semitones=0.5,
                             key_hpcp_peaks_per_frame=10, key_hpcp_num_harmonics=6),
    "bass_heavy": dict(enable_key_hpcp_bass_blend=1, key_hpcp_bass_weight=0.9, key_hpcp_bass_fmin_hz=40.0,
                       key_hpcp_bass_fmax_hz=500.0, key_hpcp_peaks_per_frame=30),
    "log_frequency": dict(enable_key_log_frequency=1),
    "log_frequency_tuning": dict(enable_key_log_frequency=1, enable_key_tuning_compensation=1),
    "beat_sync": dict(enable_key_beat_synchronous=1),
    "beat_sync_tuned_hard": dict(enable_key_beat_synchronous=1, enable_key_tuning_compensation=1,
                                 key_tuning_max_abs_semitones=0.5, soft_chroma_mapping=0),
    "beat_sync_log": dict(enable_key_beat_synchronous=1, enable_key_log_frequency=1),
    "key_hpss": dict(enable_key_hpss_harmonic=1),
    "key_hpss_small": dict(enable_key_hpss_harmonic=1, key_hpss_frame_step=1, key_hpss_time_margin=3,
                           key_hpss_freq_margin=5, key_hpss_mask_power=1.0),
    "key_hpss_wide": dict(enable_key_hpss_harmonic=1, key_hpss_frame_step=3, key_hpss_time_margin=12,
                          key_hpss_freq_margin=16, key_hpss_mask_power=3.0, enable_key_hpcp=0),
    "beat_sync_no_voting": dict(enable_key_beat_synchronous=1, enable_key_segment_voting=0,
                                chroma_sharpening_power=2.0),
}


def _run(case, xs, sr=SR):
    cfg = sdsp.default_config()
    ocfg = oracle.default_config()
    for k, v in CASES[case].items():
        setattr(cfg, k, v)
        setattr(ocfg, k, v)
    got = sdsp.analyze_batch(xs, sr, cfg)
    refs = []
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, sr, ocfg)
        assert st == 0, (case, i, ref)
        assert not isinstance(got[i], Exception), (case, i, got[i])
        bad = parity.diff_results(got[i], ref)
        assert not bad, f"{case} track {i}: {bad}"
        assert parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, (case, i)
        refs.append(ref)
    return got, refs


@pytest.mark.parametrize("case", sorted(CASES))
def test_chroma_option_parity(case):
    _run(case, tracks())


@pytest.mark.parametrize("sr", [22050, 48000])
@pytest.mark.parametrize("case", ["plain_soft", "tuning_hpcp_wide", "log_frequency", "bass_white_tuned", "beat_sync",
                                  "key_hpss"])
def test_chroma_option_sample_rates(case, sr):
    xs = [synth.make_track(s, seconds=20.0, sr=sr)[0] for s in (5, 7)]
    _run(case, xs, sr)


def test_beat_sync_segment_rows():
    """Beat-synchronous chroma with segments short enough that each track's beat rows make several
    segments (key_segment_len_frames is counted in beat rows there): the vote's per-track segment
    scratch is laid out in KV_ROW-float rows, so the tracks' rows must not overlap (round 6 fixed
    this path's scratch offsets, which still counted 64 floats per row)."""
    CASES["beat_sync_short_segments"] = dict(enable_key_beat_synchronous=1, key_segment_len_frames=120,
                                             key_segment_hop_frames=20)
    try:
        xs = [synth.make_track(s, seconds=sec)[0] for s, sec in ((61, 100.0), (67, 75.0), (71, 130.0))]
        got, refs = _run("beat_sync_short_segments", xs)
    finally:
        del CASES["beat_sync_short_segments"]


def test_chroma_options_change_results():
    """The front-ends are live: most cases change some key result against the default config."""
    xs = tracks()
    base = sdsp.analyze_batch(xs, SR, sdsp.default_config())
    changed = set()
    for case in ("plain_soft", "tuning_hpcp_wide", "whitening", "bass_heavy", "log_frequency", "beat_sync",
                 "time_smooth", "key_hpss"):
        cfg = sdsp.default_config()
        for k, v in CASES[case].items():
            setattr(cfg, k, v)
        for a, b in zip(sdsp.analyze_batch(xs, SR, cfg), base):
            if (a["key"], a["key_confidence"], a["key_clarity"]) != (b["key"], b["key_confidence"], b["key_clarity"]):
                changed.add(case)
    assert len(changed) >= 6, changed
