"""Pin the CPU oracle (oracle/) against fixtures generated from the reference itself.

The fixtures come from tests/golden/make_golden.py, which runs /root/reference's
own SQL generators, Params and EM loop through sqlite with Spark semantics.
"""
import math

import numpy as np
import pandas as pd
import pytest

import oracle as orc
from conftest import load_golden

PIPELINES = ["test1", "main_api_nojaro", "main_api_jaro", "test2_nulls", "synthetic_cfg1", "custom_exprs", "link_tf"]


def rel_close(a, b, tol=1e-9):
    if a is None or b is None:
        return a is None and b is None
    if isinstance(a, float) and math.isnan(a):
        return b is None or (isinstance(b, float) and math.isnan(b))
    return abs(a - b) <= tol * max(abs(a), abs(b), 1e-300)


def frame(d):
    return pd.DataFrame(d) if d else None


def pair_keys(df):
    cols = [c for c in ("_source_table_l", "unique_id_l", "_source_table_r", "unique_id_r") if c in df.columns]
    return cols


def run_oracle_pipeline(g):
    st = g["settings_completed"]
    lt = st["link_type"]
    uid = st["unique_id_column_name"]
    pairs, left, right = orc.block(st, df=frame(g.get("df")), df_l=frame(g.get("df_l")), df_r=frame(g.get("df_r")))
    cmp_df = orc.comparison_frame(pairs, left, right)
    exprs = [c["case_expression"] for c in st["comparison_columns"]]
    gam = orc.sql_gammas(cmp_df, exprs)
    names = [f"gamma_{c.get('custom_name', c.get('col_name'))}" for c in st["comparison_columns"]]
    out = pd.DataFrame({f"{uid}_l": cmp_df[f"{uid}_l"], f"{uid}_r": cmp_df[f"{uid}_r"]})
    if lt == "link_and_dedupe":
        out["_source_table_l"] = cmp_df["_source_table_l"]
        out["_source_table_r"] = cmp_df["_source_table_r"]
    for k, n in enumerate(names):
        out[n] = gam[:, k]
    keys = pair_keys(out)
    out = out.sort_values(keys + names, kind="mergesort").reset_index(drop=True)
    return out, names, cmp_df, pairs


def golden_params(g):
    st = g["settings_completed"]
    names = [f"gamma_{c.get('custom_name', c.get('col_name'))}" for c in st["comparison_columns"]]
    nlev = [c["num_levels"] for c in st["comparison_columns"]]
    lam = g["initial"]["lambda"]
    m = [g["initial"]["pi"][n]["m"] for n in names]
    u = [g["initial"]["pi"][n]["u"] for n in names]
    return names, nlev, lam, m, u, st


def test_string_values():
    g = load_golden("string_values")
    for (a, b), jw, lev in zip(g["pairs"], g["jw"], g["lev"]):
        assert orc.jaro_winkler(a, b) == jw, (a, b)
        assert orc.levenshtein(a, b) == lev, (a, b)


def test_reference_jw_examples():
    # SURVEY.md §2.3 sample values and the jar's level expectations (tests/test_spark.py:355-419)
    assert orc.jaro_winkler("smith", "smithe") == 0.9722222222222223
    assert orc.jaro_winkler("linacre", "linaker") == 0.9095238095238095
    assert orc.jaro_winkler("these strings are almost equal", "not the same at all") == 0.7009746588693956
    assert orc.jaro_winkler("", "") == 0.0


def test_case_levels():
    g = load_golden("case_levels")
    tables = {"str_comp": frame(g["str_comp"]), "float_comp": frame(g["float_comp"]), "df_names": frame(g["names"])}
    for case in g["cases"]:
        got = orc.sql_gammas(tables[case["table"]], [case["case_expression"]])[:, 0].tolist()
        assert got == case["levels"], case["name"]


@pytest.mark.parametrize("name", PIPELINES)
def test_pipeline(name):
    g = load_golden(name)
    got, names, _, _ = run_oracle_pipeline(g)
    exp = frame(g["gammas"])
    keys = pair_keys(exp)
    assert len(got) == len(exp)
    for c in keys + names:
        assert got[c].tolist() == exp[c].tolist(), c
    _check_em(g, exp[names].to_numpy(np.int8))


def _check_em(g, gam):
    names, nlev, lam, m, u, st = golden_params(g)
    if "error" in g:
        with pytest.raises(Exception):
            hist, _ = orc.em_iterate(gam, nlev, lam, m, u, st["max_iterations"], st["em_convergence"])
            orc.score(gam, nlev, hist[-1][0], hist[-1][1], hist[-1][2])
        return
    hist, mp = orc.em_iterate(gam, nlev, lam, m, u, st["max_iterations"], st["em_convergence"])
    assert len(hist) == len(g["iterations"])
    for (l2, m2, u2), it in zip(hist, g["iterations"]):
        assert rel_close(l2, it["lambda"])
        for k, n in enumerate(names):
            for a, b in zip(m2[k], it["pi"][n]["m"]):
                assert rel_close(a, b), (n, m2[k], it["pi"][n]["m"])
            for a, b in zip(u2[k], it["pi"][n]["u"]):
                assert rel_close(a, b)
    exp_mp = g["df_e"]["match_probability"]
    assert all(rel_close(float(a), b) for a, b in zip(mp, exp_mp))


def test_dgp_em():
    g = load_golden("dgp")
    names, nlev, lam, m, u, st = golden_params(g)
    gam = frame(g["df_gammas"])[names].to_numpy(np.int8)
    hist, mp = orc.em_iterate(gam, nlev, lam, m, u, st["max_iterations"], st["em_convergence"])
    assert len(hist) == len(g["iterations"])
    assert rel_close(hist[-1][0], g["iterations"][-1]["lambda"])


@pytest.mark.parametrize("case", ["link_only_plain_rules", "link_only_plain_cartesian", "link_and_dedupe_plain_rules",
                                  "link_and_dedupe_plain_cartesian", "link_only_repeat_rules",
                                  "link_only_repeat_cartesian", "link_and_dedupe_repeat_rules",
                                  "link_and_dedupe_repeat_cartesian", "dedupe_only_plain_rules",
                                  "dedupe_only_repeat_rules", "blocks_dedupe"])
def test_link_options(case):
    g = load_golden("link_options")[case]
    got, names, _, _ = run_oracle_pipeline(g)
    exp = frame(g["gammas"])
    if exp is None or len(exp) == 0:
        assert len(got) == 0
        return
    for c in pair_keys(exp) + names:
        assert got[c].tolist() == exp[c].tolist(), c
    _check_em(g, exp[names].to_numpy(np.int8))


def test_tf_adjust():
    g = load_golden("link_tf")
    df_e = frame(g["df_e"])
    tf = frame(g["df_tf"])
    lam = g["iterations"][-1]["lambda"]
    mp = df_e["match_probability"].astype(float).to_numpy()
    out, adjs = orc.tf_adjust([df_e["surname_l"].tolist()], [df_e["surname_r"].tolist()], mp, lam)
    # df_tf is sorted like df_e (same pair keys, same gamma order)
    assert tf["match_probability"].astype(float).tolist() == pytest.approx(mp.tolist(), rel=1e-12)
    exp = tf["tf_adjusted_match_prob"].astype(float).to_numpy()
    assert np.allclose(out, exp, rtol=1e-9, atol=0)
    assert np.allclose(adjs[0], tf["surname_adj"].astype(float).to_numpy(), rtol=1e-9, atol=0)
    # the vectorised restatement (the scale tests' checker) over integer value codes
    import pandas as pd
    codes, _ = pd.factorize(pd.concat([df_e["surname_l"], df_e["surname_r"]], ignore_index=True))
    n = len(df_e)
    out2, adj2 = orc.tf_adjust_codes(codes[:n], codes[n:], mp, lam)
    assert np.array_equal(out2, out, equal_nan=True)
    assert np.array_equal(adj2, adjs[0], equal_nan=True)


EDGE = ["first_estep_test1", "first_estep_nulls", "tiny_numbers_estep", "tiny_numbers_em", "ll_test1", "ll_nulls",
        "ll_cfg1", "null_uid_dedupe", "null_uid_link_and_dedupe"]


def oracle_log_likelihoods(g, gam):
    """One log-likelihood per E-step of iterate(compute_ll=True): the initial parameters, then the
    parameters after each M-step (expectation_step.py:52-57; iterate.py:45-63)."""
    names, nlev, lam, m, u, st = golden_params(g)
    hist, _ = orc.em_iterate(gam, nlev, lam, m, u, st["max_iterations"], st["em_convergence"])
    params = [(lam, m, u)] + list(hist)
    return [orc.log_likelihood(gam, nlev, *p) for p in params]


@pytest.mark.parametrize("case", EDGE)
def test_edge_cases(case):
    """Reference edge cases (tests/test_expectation.py:57-66, tests/test_nulls.py:11, tests/test_spark.py:130-160),
    NULL unique ids, and the log-likelihood of every E-step (expectation_step.py:224-272)."""
    g = load_golden("edge_cases")[case]
    got, names, _, _ = run_oracle_pipeline(g)
    exp = frame(g["gammas"])
    assert len(got) == len(exp)
    nan_none = lambda xs: [None if isinstance(v, float) and math.isnan(v) else v for v in xs]  # noqa: E731
    for c in pair_keys(exp) + names:
        assert nan_none(got[c].tolist()) == nan_none(exp[c].tolist()), c
    gam = exp[names].to_numpy(np.int8)
    _check_em(g, gam)
    if "reference_literal_mp" in g:  # the reference's own hand-calculated lists (abs 1e-8)
        assert g["df_e"]["match_probability"] == pytest.approx(g["reference_literal_mp"], abs=1e-8)
    if "log_likelihood" in g:
        lls = oracle_log_likelihoods(g, gam)
        assert len(lls) == len(g["log_likelihood"])
        for a, b in zip(lls, g["log_likelihood"]):
            assert rel_close(a, b), (a, b)


def test_histogram_em_equals_per_pair_em():
    """oracle.em_iterate_hist (the EM check of the >2^31-pair GPU test: the pattern histogram of every
    pair's comparison vector) gives the per-pair oracle's λ / m / u and match probabilities, NULL levels
    and unobserved patterns included."""
    rng = np.random.Generator(np.random.PCG64(3))
    nlev = [3, 3, 2, 2, 3]
    P = 300_001
    gam = np.stack([np.where(rng.random(P) < 0.6, 0, rng.integers(-1, L, P)) for L in nlev], 1).astype(np.int8)
    lam = 0.05
    m = [[0.1, 0.2, 0.7], [0.1, 0.3, 0.6], [0.2, 0.8], [0.3, 0.7], [0.05, 0.15, 0.8]]
    u = [[0.8, 0.15, 0.05], [0.7, 0.2, 0.1], [0.9, 0.1], [0.85, 0.15], [0.9, 0.08, 0.02]]
    h1, mp1 = orc.em_iterate(gam, nlev, lam, m, u, 6, 1e-300)
    hist = np.zeros(int(np.prod([L + 1 for L in nlev])), dtype=np.int64)
    codes = orc.pattern_codes(gam[:P // 2], nlev, hist)  # two chunks accumulate into one histogram
    codes = np.concatenate([codes, orc.pattern_codes(gam[P // 2:], nlev, hist)])
    assert hist.sum() == P and (np.bincount(codes, minlength=len(hist)) == hist).all()
    h2, mpat = orc.em_iterate_hist(hist, nlev, lam, m, u, 6, 1e-300)
    assert len(h1) == len(h2) == 6
    for (l1, m1, u1), (l2, m2, u2) in zip(h1, h2):
        assert rel_close(l1, l2)
        for a, b in zip(sum(m1, []) + sum(u1, []), sum(m2, []) + sum(u2, [])):
            assert rel_close(a, b)
    assert np.allclose(mp1, mpat[codes], rtol=1e-12, atol=0, equal_nan=True)
