"""Host fast paths of the EM loop against their plain definitions (no GPU).

quantise: `float(f"{p:.35f}")` (the reference renders m / u as 35-decimal literals, expectation_step.py:212);
f32_many: `float(np.float32(x))` per value (maximisation_step.py:19, 68-69); _copy_tree: copy.deepcopy.
"""
import copy
import math

import numpy as np

from splink_amd.engine import f32, f32_many, quantise
from splink_amd.params import _copy_tree


def test_quantise_matches_text_round_trip():
    rng = np.random.default_rng(7)
    vals = [0.0, -0.0, 1.0, 0.5, 1e-18, 9.99e-19, 1e-19, 5e-324, 1e-300, 0.1, 1 / 3, 0.9999999999999999]
    vals += rng.random(2000).tolist()
    vals += (10.0 ** rng.uniform(-40, 0, 4000)).tolist()
    vals += [v * (1 + 1e-15) for v in (1e-18, 1e-17, 3e-19)]
    for p in vals:
        want = float(f"{p:.35f}")
        got = quantise(p)
        assert got == want and math.copysign(1, got) == math.copysign(1, want), p
    assert math.isnan(quantise(float("nan")))


def test_f32_many_matches_scalar_cast():
    rng = np.random.default_rng(8)
    xs = rng.random(500).tolist() + [None, 0.0, 1.0, 1e-40, 3.4e38, None]
    assert f32_many(xs) == [f32(x) for x in xs]
    assert f32_many([]) == [] and f32_many([None]) == [None]


def test_copy_tree_is_a_deep_copy():
    tree = {"λ": 0.3, "π": {"gamma_a": {"num_levels": 3, "desc": "x", "custom": None, "flag": True,
                                        "prob_dist_match": {"level_0": {"value": 0, "probability": 0.1}},
                                        "lst": [1, 2.5, {"z": "q"}]}}}
    c = _copy_tree(tree)
    assert c == copy.deepcopy(tree)
    c["π"]["gamma_a"]["lst"][2]["z"] = "changed"
    assert tree["π"]["gamma_a"]["lst"][2]["z"] == "q"
    odd = {"v": np.float64(0.25), "t": (1, 2)}
    assert _copy_tree(odd) == odd
