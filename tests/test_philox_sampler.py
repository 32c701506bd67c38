"""Counter-based Philox random-search sampler (polytune/sampler.py): known-answer test of the generator, the
per-distribution mappings, de-duplication / space capping, and the random_search.sampler switch."""
import numpy as np
import pytest

from polyaxon_amd.polytune.sampler import PhiloxSampler, philox4x32_10, philox_random_suggestions
from polyaxon_amd.spec.hptuning import HPTuningConfig
from polyaxon_amd.spec.matrix import MatrixValidationError, parse_matrix


def test_philox_known_answers():
    # Random123 kat_vectors: philox4x32 10 rounds
    out = philox4x32_10([0], [0], [0], [0], 0, 0)
    assert [int(w[0]) for w in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    f = 0xFFFFFFFF
    out = philox4x32_10([f], [f], [f], [f], f, f)
    assert [int(w[0]) for w in out] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    out = philox4x32_10([0x243F6A88], [0x85A308D3], [0x13198A2E], [0x03707344], 0xA4093822, 0x299F31D0)
    assert [int(w[0]) for w in out] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_distributions():
    m = parse_matrix({"u": {"uniform": [2, 5]}, "lu": {"loguniform": [-3, 0]}, "n": {"normal": [1, 2]},
                      "ln": {"lognormal": [0, 0.5]}, "qu": {"quniform": [0, 10, 0.5]},
                      "v": {"values": [3, 7, 9]}, "pv": {"pvalues": [["a", 0.1], ["b", 0.6], ["c", 0.3]]}})
    s = PhiloxSampler(m)
    raw = s.draw_host(200000, seed=11)
    col = {k: raw[:, i] for i, k in enumerate(s.keys)}
    assert col["u"].min() >= 2 and col["u"].max() < 5 and abs(col["u"].mean() - 3.5) < 0.01
    assert np.exp(-3) <= col["lu"].min() and col["lu"].max() < 1 and abs(np.log(col["lu"]).mean() + 1.5) < 0.01
    assert abs(col["n"].mean() - 1) < 0.02 and abs(col["n"].std() - 2) < 0.02
    assert abs(np.log(col["ln"]).std() - 0.5) < 0.01
    assert np.allclose(col["qu"] / 0.5, np.round(col["qu"] / 0.5)) and 0 <= col["qu"].min() and col["qu"].max() <= 10
    assert set(np.unique(col["v"]).astype(int)) == {0, 1, 2}
    freq = np.bincount(col["pv"].astype(int), minlength=3) / len(raw)
    np.testing.assert_allclose(freq, [0.1, 0.6, 0.3], atol=0.01)
    rows = s.values(raw[:5])
    assert all(r["v"] in (3, 7, 9) and r["pv"] in ("a", "b", "c") for r in rows)


def test_counter_based_and_dedup():
    m = parse_matrix({"lr": {"uniform": [0, 1]}, "bs": {"values": [16, 32]}})
    a = philox_random_suggestions(m, 50, seed=3, device=None)
    b = philox_random_suggestions(m, 10, seed=3, device=None)
    assert a[:10] == b  # suggestion r does not depend on how many were drawn
    assert philox_random_suggestions(m, 10, seed=4, device=None) != b
    d = parse_matrix({"x": {"values": [1, 2, 3]}, "y": {"range": [0, 4, 1]}})
    s = philox_random_suggestions(d, 100, seed=1, device=None)
    assert len(s) == 12 and len({(r["x"], r["y"]) for r in s}) == 12  # capped at the space, no repeats
    s = philox_random_suggestions(d, 5, suggestion_params={"fixed": 1}, seed=1, device=None)
    assert all(r["fixed"] == 1 for r in s)


def test_random_search_sampler_switch():
    from polyaxon_amd.polytune.managers import RandomSearchManager

    base = {"seed": 5, "matrix": {"lr": {"loguniform": [-4, 0]}, "act": {"values": ["relu", "gelu"]}}}
    cfg = HPTuningConfig.from_dict({**base, "random_search": {"n_experiments": 6, "sampler": "device"}})
    got = RandomSearchManager(cfg).get_suggestions()
    assert got == philox_random_suggestions(cfg.matrix, 6, seed=5, device=None)
    ref = RandomSearchManager(HPTuningConfig.from_dict({**base, "random_search": {"n_experiments": 6}})).get_suggestions()
    assert len(ref) == 6 and ref != got  # the default keeps the reference's RandomState stream
    assert cfg.to_dict()["random_search"]["sampler"] == "device"
    with pytest.raises(MatrixValidationError):
        HPTuningConfig.from_dict({**base, "random_search": {"n_experiments": 6, "sampler": "gpu"}})
