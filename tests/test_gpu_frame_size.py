"""AnalysisConfig::frame_size other than 2048 and key STFT sizes other than 8192 (GPU, through
the C ABI), against the oracle.

frame_size sets the tempo path's STFT (src/lib.rs:166 -> extractor.rs:301-359: frame_size/2 + 1
bins per frame), the energy-flux onset frames (:154-159), the silence-trimming frames
(src/preprocessing/silence.rs, hop frame_size/2) and the multi-resolution STFTs
(multi_resolution.rs:237-239).  The key path has its own STFT, key_stft_frame_size /
key_stft_hop_size under enable_key_stft_override (src/lib.rs:985-1009), and without the override
reads the tempo path's spectrogram (frame_size / hop_size): the engine recomputes that one on the
key stream, bit-identical by the STFT spec.  Sizes other than the tuned 2048 / 8192 run the
general STFT kernel k_stft_gen, and every consumer of a spectrogram takes the bin count and row
stride from its frame size.  Results must equal the oracle's exactly, as for the defaults.
"""
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu

CASES = {
    "fs512_hop256": dict(frame_size=512, hop_size=256),
    "fs1024": dict(frame_size=1024),
    "fs1024_hpss": dict(frame_size=1024, enable_hpss_onsets=1),
    "fs4096": dict(frame_size=4096),
    "fs4096_hop441": dict(frame_size=4096, hop_size=441),
    "fs8192": dict(frame_size=8192),
    "key4096_hop1024": dict(key_stft_frame_size=4096, key_stft_hop_size=1024),
    "key16384": dict(key_stft_frame_size=16384),
    "key2048_hpss_mask": dict(key_stft_frame_size=2048, enable_key_hpss_harmonic=1),
    "key_no_override": dict(enable_key_stft_override=0),
    "key_no_override_fs4096": dict(enable_key_stft_override=0, frame_size=4096, hop_size=1024),
    "key4096_log_freq": dict(key_stft_frame_size=4096, enable_key_log_frequency=1),
    "key4096_tuning": dict(key_stft_frame_size=4096, enable_key_tuning_compensation=1),
}
BPMS = [62.0, 74.0, 128.0, 184.0]

_TRACKS = None


def tracks():
    global _TRACKS
    if _TRACKS is None:
        _TRACKS = [synth.make_track(700 + k, seconds=40.0, bpm=b)[0] for k, b in enumerate(BPMS)]
    return _TRACKS


def _cfg(base, opts):
    for k, v in opts.items():
        setattr(base, k, v)
    return base


@pytest.mark.parametrize("case", sorted(CASES))
def test_frame_size_parity(case):
    cfg = _cfg(sdsp.default_config(), CASES[case])
    ocfg = _cfg(oracle.default_config(), CASES[case])
    xs = tracks()
    got = sdsp.analyze_batch(xs, 44100, cfg)
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, ocfg)
        assert st == 0, (case, i, ref)
        assert not isinstance(got[i], Exception), (case, i, got[i])
        bad = parity.diff_results(got[i], ref)
        assert not bad, f"{case} track {i}: {bad}"
        assert parity.exact_fraction(got[i], ref, cfg=cfg) == 1.0, (case, i)


def test_key_stft_size_changes_results():
    """key_stft_frame_size is live: some key / key confidence differs from the 8192 default."""
    xs = tracks()
    a = sdsp.analyze_batch(xs, 44100, sdsp.default_config())
    b = sdsp.analyze_batch(xs, 44100, _cfg(sdsp.default_config(), dict(key_stft_frame_size=2048)))
    assert any((r["key"], r["key_confidence"]) != (s["key"], s["key_confidence"]) for r, s in zip(a, b))


def test_frame_size_changes_results():
    """frame_size is live: some bpm / confidence / beat grid differs from frame_size 2048."""
    xs = tracks()
    a = sdsp.analyze_batch(xs, 44100, sdsp.default_config())
    b = sdsp.analyze_batch(xs, 44100, _cfg(sdsp.default_config(), dict(frame_size=1024)))
    assert any((r["bpm"], r["bpm_confidence"], r["beat_grid"]) != (s["bpm"], s["bpm_confidence"], s["beat_grid"])
               for r, s in zip(a, b))


@pytest.mark.parametrize("fs", [1000, 32768])
def test_frame_size_refused(fs):
    """Frame sizes the engine cannot run (not a power of two in [64, 16384]) are reported per
    track as NotImplemented, not analysed with another size."""
    got = sdsp.analyze_batch(tracks()[:1], 44100, _cfg(sdsp.default_config(), dict(frame_size=fs)))
    assert isinstance(got[0], Exception)
    got = sdsp.analyze_batch(tracks()[:1], 44100, _cfg(sdsp.default_config(), dict(key_stft_frame_size=fs)))
    assert isinstance(got[0], Exception)
