"""k_features / k_mel_flux under non-default tempogram settings, GPU engine against the oracle
(bit-exact, tests/parity.py).  The kernels choose their walk per 8-bin chunk from host-built
plans (mel-free fast chunks, packed mel chunks, the general walk at band edges) and their
SuperFlux window from the configured width, so moving the mel range, the band edges and the
filter widths moves work between those paths:

* mel filterbanks with other band counts and ranges (the packed mel chunks reach into the high
  band, or shrink to a few chunks);
* band edges elsewhere (more chunks on the general walk);
* SuperFlux half widths 2 and 6 (the runtime-width kernels k_features<8,16,0> / <16,32,0>);
* mel max-filter widths other than 2 (k_mel_flux's general window).
"""
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu

CASES = {
    "mel24_50_12000": dict(tempogram_mel_n_mels=24, tempogram_mel_fmin_hz=50.0, tempogram_mel_fmax_hz=12000.0),
    "mel48_20_4000": dict(tempogram_mel_n_mels=48, tempogram_mel_fmin_hz=20.0, tempogram_mel_fmax_hz=4000.0),
    "mel_k1": dict(tempogram_mel_max_filter_bins=1),
    "mel_k3": dict(tempogram_mel_max_filter_bins=3),
    "bands_moved": dict(tempogram_band_low_max_hz=310.0, tempogram_band_mid_max_hz=2700.0,
                        tempogram_band_high_max_hz=11000.0),
    "high_to_nyquist": dict(tempogram_band_high_max_hz=0.0),
    "superflux_k2": dict(tempogram_superflux_max_filter_bins=2),
    "superflux_k6": dict(tempogram_superflux_max_filter_bins=6),
    "no_band_fusion": dict(enable_tempogram_band_fusion=0),
    "no_mel": dict(enable_tempogram_mel_novelty=0),
}

_TRACKS = None


def tracks():
    global _TRACKS
    if _TRACKS is None:
        _TRACKS = [synth.make_track(8100 + k, seconds=24.0, bpm=b)[0] for k, b in enumerate([78.0, 126.0, 171.0])]
    return _TRACKS


def _cfg(base, opts):
    for k, v in opts.items():
        setattr(base, k, v)
    return base


@pytest.mark.parametrize("case", sorted(CASES))
def test_feature_config_parity(case):
    cfg = _cfg(sdsp.default_config(), CASES[case])
    ocfg = _cfg(oracle.default_config(), CASES[case])
    xs = tracks()
    got = sdsp.analyze_batch(xs, 44100, config=cfg)
    for x, g in zip(xs, got):
        st, ref = oracle.analyze(x, 44100, ocfg)
        assert st == 0
        assert not parity.diff_results(g, ref), case
        assert parity.exact_fraction(g, ref, cfg=cfg) == 1.0, case
