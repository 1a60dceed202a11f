"""The default key path's block-folded frame energies (k_mask_rp + k_hpcp_band).

HPCP needs the masked 8192-point spectrogram only on its peak band, but folds every frame's energy
sum(x * x) over all 4,097 bins (extractor.rs:1133).  The engine's mask kernel stores the masked
values on the band only and folds each frame's squares in 64-bin blocks, HPCP folds the 65 block
sums: the one f32 sum is re-associated, every masked value and every other stage is unchanged.
The north star's tolerance (key exact, confidences within 1e-4) is what the key fields are held to;
every other field stays bit-identical to the oracle.  The config-2 golden (64 x 3-min) is checked
the same way in test_gpu_batch_paths.py.
"""
import numpy as np
import pytest

import oracle
import parity
import sdsp
import synth

pytestmark = pytest.mark.gpu


def _tracks():
    xs = [synth.make_track(9100 + k, seconds=20.0 + 7 * (k % 9), mode=k % 2, tonic=(5 * k) % 12)[0] for k in range(40)]
    xs += [synth.make_track(9200 + k, seconds=180.0)[0] for k in range(4)]
    return xs


def test_block_energies_key_exact_fields_bitexact():
    xs = _tracks()
    got = sdsp.analyze_batch(xs)
    n_key_bits = 0
    worst = 0.0
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100)
        assert st == 0, i
        assert got[i]["key"] == ref["key"], (i, got[i]["key"], ref["key"])
        assert not parity.diff_results(got[i], ref), (i, parity.diff_results(got[i], ref))
        g, e = parity.result_digest(got[i]), parity.result_digest(ref)
        assert all(g[k] == e[k] for k in g if k not in parity.KEY_ENERGY_FIELDS), i
        n_key_bits += int(all(g[k] == e[k] for k in parity.KEY_ENERGY_FIELDS))
        worst = max(worst, abs(got[i]["key_confidence"] - ref["key_confidence"]),
                    abs(got[i]["key_clarity"] - ref["key_clarity"]))
    print(f"key-energy fields bit-equal on {n_key_bits} of {len(xs)} tracks; worst |diff| {worst:.3g}")
    assert worst <= parity.TOL


def test_exact_energy_configs_stay_bitexact():
    """Configurations the band path does not serve keep k_mask_r + the full-spectrum HPCP walk,
    bit-identical to the oracle in every field (here: a mask margin other than 12)."""
    cfg = sdsp.default_config()
    cfg.key_spectrogram_smooth_margin = 8
    xs = [synth.make_track(9300 + k, seconds=25.0 + 4 * k)[0] for k in range(4)]
    got = sdsp.analyze_batch(xs, config=cfg)
    for i, x in enumerate(xs):
        st, ref = oracle.analyze(x, 44100, config=cfg)
        assert st == 0 and parity.exact_fraction(got[i], ref, strict=True) == 1.0, i

