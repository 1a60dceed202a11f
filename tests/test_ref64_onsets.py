"""The CPU restatement's onset stages (oracle/o_onset.cpp: energy flux, spectral flux, HFC, the
consensus vote) against an independent float64 reading of the same Rust (tests/ref64.py:
energy_flux_onsets, spectral_flux_onsets, hfc_onsets, vote_onsets, consensus_onsets), SURVEY §8a
rows a4, a6, a7, a8.  CPU only.

References: src/features/onset/energy_flux.rs:67-243, spectral_flux.rs:69-221, hfc.rs:76-214,
consensus.rs:111-287 and their call site src/lib.rs:152-289.  The float64 reading takes the trimmed,
normalised samples and the spec-pinned hop-512 STFT magnitudes; the oracle's per-detector onset
lists come from its trace.  Lists are compared exactly (they are integer sample positions); a peak
decision whose two sides differ by less than 1e-6 of the curve's maximum is left to the
reference's f32 rounding (ref64 records it), and the list is then compared except at that peak.
The consensus (the onsets the beat tracker receives) is compared exactly when no detector list
holds such a near tie.
"""
import os

import numpy as np
import pytest

import oracle
import parity
import ref64
import synth

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = ["120bpm_4bar.wav", "128bpm_4bar.wav", "cmajor_scale.wav", "mixed_silence.wav"]
SYNTH = [(s, (20.0, 30.0, 45.0)[s % 3]) for s in range(16)]
CASES = [("fixture", n) for n in FIXTURES] + [("synth", s) for s in SYNTH]
_cache = {}


def _run(kind, what):
    key = (kind, str(what))
    if key not in _cache:
        if kind == "fixture":
            x, sr = parity.load_wav(os.path.join(HERE, "golden", what))
        else:
            x, *_ = synth.make_track(what[0], seconds=what[1])
            sr = 44100
        st, r, tr = oracle.analyze(x, sr, trace=True)
        assert st == 0, r
        _, xn = oracle.normalize(x, 0, sr)
        xt = xn[tr["trim_start"]:tr["trim_end"]]
        mags = oracle.stft(xt, 2048, 512).astype(np.float64)
        ties = ref64.Ties()
        got = ref64.consensus_onsets(xt, sr, mags, ties=ties)
        _cache[key] = (tr, got, list(ties))
    return _cache[key]


def _tie_positions(ties, tag, hop=512, frames=True):
    """sample positions of the peaks a near tie touches (either side of the comparison)"""
    return [t for t in ties if t[0] == tag]


def _compare(a, b, tied):
    a, b = list(a), list(b)
    if not tied:
        assert a == b
        return
    # a near tie can add or drop the one peak it decides: at most one difference per tie
    diff = set(a) ^ set(b)
    assert len(diff) <= len(tied), (sorted(diff), len(tied))


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_onset_lists(kind, what):
    tr, (energy, spectral, hfc, chosen), ties = _run(kind, what)
    _compare(tr["energy_onsets"], energy, _tie_positions(ties, "energy-peak"))
    _compare(tr["spectral_onsets"], spectral, _tie_positions(ties, "spectral-peak"))
    _compare(tr["hfc_onsets"], hfc, _tie_positions(ties, "hfc-peak"))
    if not ties:
        assert list(tr["chosen_onsets"]) == list(chosen)


def test_onset_coverage():
    """The detectors find onsets on the rhythmic inputs, the consensus keeps strong (>= 2 method)
    onsets, and near ties are rare."""
    n_tie = 0
    for kind, what in CASES:
        tr, (energy, spectral, hfc, chosen), ties = _run(kind, what)
        n_tie += bool(ties)
        if kind == "synth":
            assert len(energy) > 4 and len(spectral) > 4 and len(hfc) > 4 and len(chosen) > 4
    assert n_tie <= 0.2 * len(CASES), n_tie


def test_vote_onsets_known_answers():
    """ref64.vote_onsets against the reference's own consensus unit tests (consensus.rs:293-477,
    restated one for one; lists are (energy, spectral, hfc, hpss))."""
    v = ref64.vote_onsets
    q = (0.25, 0.25, 0.25, 0.25)
    c = v([[1000], [1000], [1000], [1000]], q, 50, 44100)  # test_consensus_voting_basic
    assert len(c) == 1 and c[0][0] == 1000 and c[0][2] == 4 and abs(c[0][1] - 1.0) < 0.01
    c = v([[1000], [1050], [980], [1020]], q, 50, 44100)  # _clustering
    assert len(c) == 1 and c[0][2] == 4 and abs(c[0][1] - 1.0) < 0.01
    c = v([[1000, 50000], [1050, 50500], [980, 50200], [1020, 49900]], q, 50, 44100)  # _separate_onsets
    assert len(c) == 2 and c[0][2] == 4 and c[1][2] == 4
    c = v([[1000], [1050], [], []], (0.3, 0.3, 0.2, 0.2), 50, 44100)  # _partial_agreement
    assert len(c) == 1 and c[0][2] == 2 and abs(c[0][1] - 0.6) < 0.01
    c = v([[1000], [], [], []], (0.5, 0.2, 0.2, 0.1), 50, 44100)  # _weighted
    assert len(c) == 1 and c[0][2] == 1 and abs(c[0][1] - 0.5) < 0.01
    assert v([[], [], [], []], q, 50, 44100) == []  # _empty
    c = v([[1000, 20000, 50000], [1050, 20050, 50500], [980, 20100], [1020, 19950]], q, 50, 44100)  # _sorted_by_confidence
    assert len(c) >= 2 and c[0][2] == 4
    assert all(c[i][1] <= c[i - 1][1] for i in range(1, len(c)))


_cache64 = {}


def _run64(kind, what):
    """_run's float64 reading from a front end sharing nothing with the CPU restatement but the trim
    bounds (ref64.normalize_peak64, ref64.stft64)."""
    key = (kind, str(what))
    if key not in _cache64:
        tr = _run(kind, what)[0]
        if kind == "fixture":
            x, sr = parity.load_wav(os.path.join(HERE, "golden", what))
        else:
            x, *_ = synth.make_track(what[0], seconds=what[1])
            sr = 44100
        xt = ref64.normalize_peak64(x)[tr["trim_start"]:tr["trim_end"]]
        ties = ref64.Ties()
        got = ref64.consensus_onsets(xt, sr, ref64.stft64(xt, 2048, 512), ties=ties)
        _cache64[key] = (tr, got, list(ties))
    return _cache64[key]


@pytest.mark.parametrize("kind,what", CASES, ids=[f"{k}-{w}" for k, w in CASES])
def test_onset_lists_float64_front_end(kind, what):
    """The onset lists from the float64 front end against the oracle's, with the near-tie rule of
    test_onset_lists (the energy, spectral-flux and HFC lists and the consensus)."""
    tr, (energy, spectral, hfc, chosen), ties = _run64(kind, what)
    _compare(tr["energy_onsets"], energy, _tie_positions(ties, "energy-peak"))
    _compare(tr["spectral_onsets"], spectral, _tie_positions(ties, "spectral-peak"))
    _compare(tr["hfc_onsets"], hfc, _tie_positions(ties, "hfc-peak"))
    if not ties:
        assert list(tr["chosen_onsets"]) == list(chosen)

