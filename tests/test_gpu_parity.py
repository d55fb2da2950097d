"""Parity of the HIP path (through the C ABI) with the reference goldens and the CPU oracle."""
import copy
import math
import warnings

import numpy as np
import pandas as pd
import pytest

import oracle as orc
from conftest import load_golden

pytestmark = pytest.mark.gpu
warnings.filterwarnings("ignore")

PIPELINES = ["test1", "main_api_nojaro", "main_api_jaro", "test2_nulls", "synthetic_cfg1", "custom_exprs", "link_tf"]
LINK_CASES = ["link_only_plain_rules", "link_only_plain_cartesian", "link_and_dedupe_plain_rules",
              "link_and_dedupe_plain_cartesian", "link_only_repeat_rules", "link_only_repeat_cartesian",
              "link_and_dedupe_repeat_rules", "link_and_dedupe_repeat_cartesian", "dedupe_only_plain_rules",
              "dedupe_only_repeat_rules", "blocks_dedupe"]


@pytest.fixture(scope="module")
def amd():
    from splink_amd import AmdSession, _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    return AmdSession(0)


def spark_for(jaro, amd):
    return amd if jaro else "supress_warnings"


def frame(d):
    return pd.DataFrame(d) if d else None


def rel_close(a, b, tol=1e-9):
    """Relative closeness; NULL (None) and NaN are the same missing value."""
    a = None if (isinstance(a, float) and math.isnan(a)) else a
    b = None if (isinstance(b, float) and math.isnan(b)) else b
    if a is None or b is None:
        return a is None and b is None
    return abs(a - b) <= tol * max(abs(a), abs(b), 1e-300)


def sort_like_golden(df):
    keys = [k for k in ("_source_table_l", "unique_id_l", "_source_table_r", "unique_id_r") if k in df.columns]
    rest = [c for c in df.columns if c.startswith("gamma_")]
    return df.sort_values(keys + rest, kind="mergesort").reset_index(drop=True)


def compare_frames(got: pd.DataFrame, exp: dict, columns):
    assert list(got.columns) == list(columns)
    got = sort_like_golden(got)
    for c in columns:
        gv, ev = got[c].tolist(), exp[c]
        assert len(gv) == len(ev), c
        for a, b in zip(gv, ev):
            if isinstance(b, float) or (isinstance(a, float) and not isinstance(b, str)):
                a = None if a is None else float(a)
                assert rel_close(a, b), (c, a, b)
            else:
                if isinstance(a, float) and math.isnan(a):
                    a = None
                assert a == b, (c, a, b)


def check_history(params, g):
    if not g["iterations"]:  # max_iterations = 0: the initial parameters, untouched
        assert params.param_history == []
        assert rel_close(params.params["λ"], g["initial"]["lambda"])
        return
    hist = params.param_history[1:] + [params.params]
    assert len(hist) == len(g["iterations"])
    for p, it in zip(hist, g["iterations"]):
        assert rel_close(p["λ"], it["lambda"])
        for gname, d in it["pi"].items():
            for i, (m, u) in enumerate(zip(d["m"], d["u"])):
                assert rel_close(p["π"][gname]["prob_dist_match"][f"level_{i}"]["probability"], m), (gname, i)
                assert rel_close(p["π"][gname]["prob_dist_non_match"][f"level_{i}"]["probability"], u), (gname, i)


def run_linker(g, amd):
    from splink_amd import Splink
    settings = copy.deepcopy(g["settings_in"])
    linker = Splink(settings, spark_for(g["jaro"], amd), df=frame(g.get("df")), df_l=frame(g.get("df_l")),
                    df_r=frame(g.get("df_r")))
    return linker


@pytest.mark.parametrize("name", PIPELINES)
def test_pipeline_matches_reference(name, amd):
    g = load_golden(name)
    linker = run_linker(g, amd)
    if "error" in g:
        with pytest.raises(Exception):
            linker.get_scored_comparisons().toPandas()
        return
    df_e = linker.get_scored_comparisons()
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])
    check_history(linker.params, g)
    if "df_tf" in g:
        tf = linker.make_term_frequency_adjustments(df_e).toPandas()
        compare_frames(tf, g["df_tf"], g["df_tf_columns"])


def test_tf_host_value_ids_match_device_ids(amd):
    """The tf adjustment keyed by the device dictionary ids (default) and by host-factorised values
    (the path for columns the job did not decode on the device) give the reference golden."""
    g = load_golden("link_tf")
    for host_ids in (False, True):
        linker = run_linker(g, amd)
        df_e = linker.get_scored_comparisons()
        job, saved = df_e.job, df_e.job._col_index
        if host_ids:  # hide the device-decoded columns from the tf stage only
            job._col_index = {k: v for k, v in saved.items() if k[1] != "str"}
        tf_frame = linker.make_term_frequency_adjustments(df_e)
        job._col_index = saved
        tf = tf_frame.toPandas()
        compare_frames(tf, g["df_tf"], g["df_tf_columns"])


@pytest.mark.parametrize("case", LINK_CASES)
def test_link_options_match_reference(case, amd):
    g = load_golden("link_options")[case]
    linker = run_linker(g, amd)
    if "error" in g:
        with pytest.raises(Exception):
            linker.get_scored_comparisons().toPandas()
        return
    df_e = linker.get_scored_comparisons()
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])
    check_history(linker.params, g)


def test_em_from_gamma_table(amd):
    from splink_amd.iterate import iterate
    from splink_amd.params import Params
    g = load_golden("dgp")
    settings = copy.deepcopy(g["settings_in"])
    params = Params(settings, "supress_warnings")
    df_e = iterate(frame(g["df_gammas"]), params, params.settings, "supress_warnings")
    check_history(params, g)
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])


def test_case_levels(amd):
    from splink_amd.gammas import add_gammas
    g = load_golden("case_levels")
    tables = {"str_comp": frame(g["str_comp"]), "float_comp": frame(g["float_comp"]), "df_names": frame(g["names"])}
    for case in g["cases"]:
        t = tables[case["table"]]
        st = {"link_type": "dedupe_only", "comparison_columns": [
            {"custom_name": "x", "custom_columns_used": ["a"], "num_levels": 4,
             "case_expression": case["case_expression"]}]}
        gf = add_gammas(t, st, amd)
        got = gf.gamma_matrix()[:, 0].tolist()
        assert got == case["levels"], case["name"]


def test_udf_exact_values(amd):
    from splink_amd import _native as N
    g = load_golden("string_values")
    ctx = N.Context(0)
    left = [a for a, b in g["pairs"]]
    right = [b for a, b in g["pairs"]]
    jw = ctx.jaro_winkler_sim(left, right)
    lev = ctx.levenshtein(left, right)
    for i, (a, b) in enumerate(g["pairs"]):
        assert jw[i] == g["jw"][i], (a, b, jw[i], g["jw"][i])  # bit-exact fp64
        assert lev[i] == g["lev"][i], (a, b)


def test_udf_long_and_surrogate_strings(amd):
    from splink_amd import _native as N
    rng = np.random.Generator(np.random.PCG64(7))
    alpha = list("abcdefgh") + ["é", "\U0001F600", "\U0001D400"]
    left, right = [], []
    for n in (0, 1, 39, 40, 41, 63, 64, 65, 100, 300, 500):  # <= 1000 UTF-16 units with surrogate pairs
        for _ in range(8):
            a = "".join(rng.choice(alpha, size=n))
            b = "".join(rng.choice(alpha, size=max(0, n + int(rng.integers(-5, 6)))))
            left.append(a)
            right.append(b)
    ctx = N.Context(0)
    jw, lev = ctx.jaro_winkler_sim(left, right), ctx.levenshtein(left, right)
    for i in range(len(left)):
        assert jw[i] == orc.jaro_winkler(left[i], right[i])
        assert lev[i] == orc.levenshtein(left[i], right[i])


def _long_pairs(seed, lengths, reps):
    rng = np.random.Generator(np.random.PCG64(seed))
    alpha = list("abcdefgh") + ["é", "\U0001F600"]
    left, right = [], []
    for n in lengths:
        for r in range(reps):
            a = "".join(rng.choice(alpha, size=n))
            b = _mutate(rng, a, int(rng.integers(0, 12)), alpha) if r % 2 == 0 else "".join(rng.choice(alpha, size=n))
            left.append(a)
            right.append(b)
    return left, right


def test_strings_past_slow_limit(amd):
    """Strings longer than the slow pass's 1024-unit scratch arrays (up to 6000 UTF-16 units, with
    surrogate pairs) go through the huge pass (device scratch sized to the longest row): the bulk UDFs
    and the comparison levels of template Jaro-Winkler / Levenshtein columns and of a general program
    agree with the oracle.  Spark compares strings of any length; there is no limit to hit."""
    from splink_amd import _native as N
    from splink_amd.gammas import add_gammas
    left, right = _long_pairs(41, [700, 1023, 1024, 1025, 1600, 3000], 4)
    left += ["x" * 5000, "ab" * 3000, "short"]
    right += ["x" * 4990 + "y", "ab" * 2990, "é" * 2000]
    ctx = N.Context(0)
    jw, lev = ctx.jaro_winkler_sim(left, right), ctx.levenshtein(left, right)
    ref_jw = [orc.jaro_winkler(a, b) for a, b in zip(left, right)]
    ref_lev = [orc.levenshtein(a, b) for a, b in zip(left, right)]
    for i in range(len(left)):
        assert jw[i] == ref_jw[i], (len(left[i]), len(right[i]), jw[i], ref_jw[i])
        assert lev[i] == ref_lev[i], (len(left[i]), len(right[i]))
    df = pd.DataFrame({"a_l": left + [None], "a_r": right + ["x"]})
    lev_lv = ("case when a_l is null or a_r is null then -1 "
              + " ".join(f"when levenshtein(a_l, a_r) <= {d} then {5 - k}" for k, d in enumerate((0, 5, 20, 200, 1000)))
              + " else 0 end")
    jw_lv = ("case when a_l is null or a_r is null then -1 when jaro_winkler_sim(a_l, a_r) >= 0.97 then 3 "
             "when jaro_winkler_sim(a_l, a_r) >= 0.9 then 2 when jaro_winkler_sim(a_l, a_r) >= 0.7 then 1 else 0 end")
    mixed = ("case when a_l is null or a_r is null then -1 "
             "when jaro_winkler_sim(a_l, a_r) >= 0.9 and levenshtein(a_l, a_r) <= 300 then 2 "
             "when length(a_l) > 1024 or levenshtein(a_l, a_r) <= 1000 then 1 else 0 end")
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "lv", "custom_columns_used": ["a"], "num_levels": 6, "case_expression": lev_lv,
         "m_probabilities": [0.1, 0.1, 0.1, 0.1, 0.2, 0.4], "u_probabilities": [0.5, 0.2, 0.1, 0.1, 0.05, 0.05]},
        {"custom_name": "jw", "custom_columns_used": ["a"], "num_levels": 4, "case_expression": jw_lv},
        {"custom_name": "mx", "custom_columns_used": ["a"], "num_levels": 3, "case_expression": mixed}]}
    got = add_gammas(df, st, amd).gamma_matrix()
    for i, (a, b) in enumerate(zip(left, right)):
        d, j = ref_lev[i], ref_jw[i]
        want_lv = next((5 - k for k, t in enumerate((0, 5, 20, 200, 1000)) if d <= t), 0)
        want_jw = 3 if j >= 0.97 else 2 if j >= 0.9 else 1 if j >= 0.7 else 0
        want_mx = 2 if (j >= 0.9 and d <= 300) else 1 if (len(a) > 1024 or d <= 1000) else 0
        assert list(got[i]) == [want_lv, want_jw, want_mx], (i, len(a), len(b), d, j, list(got[i]))
    assert list(got[-1]) == [-1, -1, -1]


def test_levenshtein_cut_around_thresholds(amd):
    """The exact passes stop a scan once the end cell's diagonal exceeds the largest distance any test can
    still pass (the cut).  Pairs whose distance straddles that cut -- 0 to 0.7 x length edits, insertion-
    and deletion-heavy so the lengths differ, rows of 20-128 units through every word width, free text
    and a four-letter alphabet -- must give the reference's levels for ratio tests at 0.2 / 0.3 / 0.4 and
    absolute tests at 3 / 9 / 20."""
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(77))
    alphas = [list("abcd"), list("abcdefghijklmnopqrstuvwxyz0123456789 ,.")]
    left, right = [], []
    for n in (20, 31, 33, 45, 63, 64, 66, 90, 127, 128):
        for alpha in alphas:
            for frac in (0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.7):
                for _ in range(3):
                    a = "".join(rng.choice(alpha, size=n))
                    b = list(a)
                    for _e in range(int(round(frac * n))):
                        op = int(rng.integers(4))
                        i = int(rng.integers(len(b) + 1))
                        if op <= 1 and len(b) < 128:
                            b.insert(i, alpha[int(rng.integers(len(alpha)))])
                        elif op == 2 and b:
                            del b[min(i, len(b) - 1)]
                        elif b:
                            b[min(i, len(b) - 1)] = alpha[int(rng.integers(len(alpha)))]
                    left.append(a)
                    right.append("".join(b))
    ratio = "levenshtein(a_l, a_r)/((length(a_l) + length(a_r))/2)"
    lr = ("case when a_l is null or a_r is null then -1 when a_l = a_r then 3 "
          f"when {ratio} <= 0.2 then 2 when {ratio} <= 0.3 then 1 when {ratio} <= 0.4 then 0 else 0 end")
    la = ("case when a_l is null or a_r is null then -1 when levenshtein(a_l, a_r) <= 3 then 3 "
          "when levenshtein(a_l, a_r) <= 9 then 2 when levenshtein(a_l, a_r) <= 20 then 1 else 0 end")
    df = pd.DataFrame({"a_l": left, "a_r": right})
    mu = {"m_probabilities": [0.1, 0.2, 0.3, 0.4], "u_probabilities": [0.4, 0.3, 0.2, 0.1]}
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "lr", "custom_columns_used": ["a"], "num_levels": 4, "case_expression": lr, **mu},
        {"custom_name": "la", "custom_columns_used": ["a"], "num_levels": 4, "case_expression": la, **mu}]}
    gf = add_gammas(df, st, amd)
    got = gf.gamma_matrix()
    for i, (a, b) in enumerate(zip(left, right)):
        d = orc.levenshtein(a, b)
        r = d / ((len(a) + len(b)) / 2)
        want_r = 3 if a == b else 2 if r <= 0.2 else 1 if r <= 0.3 else 0
        want_a = 3 if d <= 3 else 2 if d <= 9 else 1 if d <= 20 else 0
        assert list(got[i]) == [want_r, want_a], (len(a), len(b), d, r, list(got[i]))
    # every Levenshtein kernel mode (per lane, lane refill, refill in free-text columns, no bag decisions) is
    # held to the same cut-edge cells
    _lev_variants_agree(gf.job, gf.settings, got)


def test_levenshtein_band_widths(amd):
    """Rows of 65-128 units run the slow pass's banded scan (diagonals [-(cut - dm) / 2, (cut + dm) / 2] in one
    word) when every lane's band fits: a ratio cut at 0.2 (bands of <= 32 diagonals), at 0.45 (33-64), and an
    absolute cut of 75 (bands past 64: the 128-bit scan).  Distances straddle each cut, the lengths differ by
    up to the cut, and some pairs share long prefixes / suffixes (the band then covers a stripped remainder of
    <= 64 units).  Levels against the oracle's Levenshtein, in every kernel mode."""
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(65))
    alphas = [list("ab"), list("abcdefghijklmnopqrstuvwxyz0123456789 ,.")]
    left, right = [], []
    for n in (65, 70, 81, 96, 110, 127, 128):
        for alpha in alphas:
            for frac in (0.05, 0.15, 0.2, 0.25, 0.4, 0.45, 0.5, 0.6, 0.75, 0.9):
                for rep in range(4):
                    a = "".join(rng.choice(alpha, size=n))
                    b = list(a)
                    lo, hi = (0, len(b)) if rep < 3 else (n // 3, 2 * n // 3)  # rep 3: edits in the middle third
                    for _e in range(int(round(frac * n))):
                        op = int(rng.integers(3 if rep != 1 else 2))  # rep 1: no deletions (length gaps)
                        i = int(rng.integers(lo, min(hi, len(b)) + 1))
                        if op == 0 and len(b) < 128:
                            b.insert(i, alpha[int(rng.integers(len(alpha)))])
                        elif op == 2 and len(b) > 1:
                            del b[min(i, len(b) - 1)]
                        elif b:
                            b[min(i, len(b) - 1)] = alpha[int(rng.integers(len(alpha)))]
                    left.append(a)
                    right.append("".join(b))
    ratio = "levenshtein(a_l, a_r)/((length(a_l) + length(a_r))/2)"
    r2 = ("case when a_l is null or a_r is null then -1 when a_l = a_r then 2 "
          f"when {ratio} <= 0.2 then 1 else 0 end")
    r45 = ("case when a_l is null or a_r is null then -1 when a_l = a_r then 3 "
           f"when {ratio} <= 0.3 then 2 when {ratio} <= 0.45 then 1 else 0 end")
    a75 = ("case when a_l is null or a_r is null then -1 when levenshtein(a_l, a_r) <= 10 then 3 "
           "when levenshtein(a_l, a_r) <= 40 then 2 when levenshtein(a_l, a_r) <= 75 then 1 else 0 end")
    df = pd.DataFrame({"a_l": left, "a_r": right})
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "r2", "custom_columns_used": ["a"], "num_levels": 3, "case_expression": r2},
        {"custom_name": "r45", "custom_columns_used": ["a"], "num_levels": 4, "case_expression": r45},
        {"custom_name": "a75", "custom_columns_used": ["a"], "num_levels": 4, "case_expression": a75}]}
    gf = add_gammas(df, st, amd)
    got = gf.gamma_matrix()
    for i, (a, b) in enumerate(zip(left, right)):
        d = orc.levenshtein(a, b)
        r = d / ((len(a) + len(b)) / 2)
        want = [2 if a == b else 1 if r <= 0.2 else 0,
                3 if a == b else 2 if r <= 0.3 else 1 if r <= 0.45 else 0,
                3 if d <= 10 else 2 if d <= 40 else 1 if d <= 75 else 0]
        assert list(got[i]) == want, (len(a), len(b), d, r, list(got[i]))
    _lev_variants_agree(gf.job, gf.settings, got)


def test_fused_jw_slow_lists_of_one_pair(amd):
    """Two Jaro-Winkler columns share one exact launch and one slow-list launch (k_gamma_slow over both lists).
    When BOTH of a pair's cells are past the exact pass's 64 units they are on both slow lists, and the two
    columns' adds to the pair's one packed code must not race (round 6: they were plain read-modify-writes).
    Every pair here has long, similar first names and surnames, so most cells of both columns take the slow
    lists; the codes must match the oracle's comparison vectors exactly."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    rng = np.random.Generator(np.random.PCG64(91))
    n = 360
    base_f, base_s = "Maximiliana-Theodora-" * 3, "Vanderbilt-Oosterhuizen-" * 3

    def noisy(base):
        s = list(base + "".join(rng.choice(list("abcdefgh"), 6)))
        for _ in range(int(rng.integers(0, 6))):
            s[int(rng.integers(len(s)))] = str(rng.choice(list("xyzqw")))
        return "".join(s)

    df = pd.DataFrame({"unique_id": np.arange(n), "first_name": [noisy(base_f) for _ in range(n)],
                       "surname": [noisy(base_s) for _ in range(n)]})
    st = complete_settings_dict({"link_type": "dedupe_only", "blocking_rules": [],
                                 "comparison_columns": [{"col_name": "first_name", "num_levels": 3},
                                                        {"col_name": "surname", "num_levels": 3}]}, amd)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block([])
    job.gammas(st)
    got = job.gammas_host()
    l, r = job.pair_rows()
    t = job.tables[0]
    cols = [orc.StrCol(t[c].tolist()) for c in ("first_name", "surname")]
    want = orc.template_gammas([("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88])], cols, cols, l, r)
    assert len(got) == n * (n - 1) // 2
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert len(bad) == 0, (len(bad), got[bad[:5]], want[bad[:5]])


def test_jw_filter_field_edges(amd):
    """The filter bounds a Jaro-Winkler column from the row image's fields: the sketch (matches) and the
    four head units (the Winkler prefix, which this jar does not cap at four).  Pairs at those edges --
    shared prefixes of 0-5 units, units equal in their low byte ('a' U+0061 / 'Š' U+0160, 'b' / 'ţ'
    U+0163), lengths 1-20 and 250-300 -- must give the reference's levels at thresholds on either side
    of their similarities."""
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(11))
    alpha = list("abcdefghij")
    left, right = [], []
    for n in (1, 2, 3, 4, 5, 6, 8, 11, 12, 20):
        for pre in range(0, 6):
            for _ in range(6):
                a = "".join(rng.choice(alpha, size=n))
                tail = "".join(rng.choice(alpha, size=max(0, n + int(rng.integers(-2, 3)) - min(pre, n))))
                left.append(a)
                right.append(a[:pre] + tail)
    for a, b in (("abcd", "Šbcd"), ("abcdx", "Šbcdy"), ("abba", "aţba"), ("abcdefghijk", "abcŠefghijk"),
                 ("Šţa", "abŠ"), ("ab", "Šţ"), ("aaaa", "aaaŠ")):
        left.append(a)
        right.append(b)
    for n in (250, 252, 253, 254, 255, 256, 258, 300):
        for r in range(4):
            a = "".join(rng.choice(alpha, size=n))
            b = _mutate(rng, a, int(rng.integers(1, 6)), alpha) if r % 2 == 0 else a[:n - 1] + "z"
            left.append(a)
            right.append(b)
    ref = [orc.jaro_winkler(a, b) for a, b in zip(left, right)]
    ts = (0.98, 0.94, 0.9, 0.85, 0.8, 0.7)
    jw_lv = ("case when a_l is null or a_r is null then -1 "
             + " ".join(f"when jaro_winkler_sim(a_l, a_r) >= {t} then {len(ts) - k}" for k, t in enumerate(ts))
             + " else 0 end")
    df = pd.DataFrame({"a_l": left, "a_r": right})
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "jw", "custom_columns_used": ["a"], "num_levels": len(ts) + 1, "case_expression": jw_lv,
         "m_probabilities": [0.05, 0.05, 0.1, 0.1, 0.1, 0.2, 0.4], "u_probabilities": [0.4, 0.2, 0.1, 0.1, 0.1, 0.05, 0.05]}]}
    got = add_gammas(df, st, amd).gamma_matrix()[:, 0]
    for i, j in enumerate(ref):
        want = next((len(ts) - k for k, t in enumerate(ts) if j >= t), 0)
        assert got[i] == want, (left[i], right[i], j, got[i])


def _synthetic(n, seed, **kw):
    from splink_amd.synthetic import make_records
    return make_records(n, seed=seed, **kw)[["unique_id", "first_name", "surname", "dob", "city", "email"]]


def _pandas_block(df, rules, uid="unique_id"):
    """Independent equi-join restatement with pandas merges (hash joins)."""
    seen = None
    out = []
    for cols in rules:
        l = df.dropna(subset=cols).reset_index().rename(columns={"index": "row"})
        m = l.merge(l, on=cols, suffixes=("_l", "_r"))
        m = m[m[f"{uid}_l"] < m[f"{uid}_r"]]
        pairs = set(zip(m["row_l"].to_numpy(), m["row_r"].to_numpy()))
        if seen is not None:
            pairs -= seen
        out.append(pairs)
        seen = pairs if seen is None else seen | pairs
    allp = set().union(*out)
    return np.array(sorted(allp), dtype=np.int64).reshape(-1, 2)


@pytest.mark.parametrize("shards", [1, 3])
def test_blocking_and_gammas_at_scale(amd, shards):
    from splink_amd.engine import Job
    from splink_amd.synthetic import cfg_settings
    from splink_amd.settings import complete_settings_dict
    df = _synthetic(30000, seed=11, surname_vocab=800, first_vocab=400, city_vocab=100)
    st = complete_settings_dict(cfg_settings(2), amd)
    rows = []
    codes = []
    table = None
    for s in range(shards):
        job = Job("dedupe_only", [df], "unique_id", 0, shard=(s, shards))
        job.block(st["blocking_rules"])
        if table is None:
            table = job.tables[0]  # pair rows index the job's blocking-key clustered table
            assert sorted(table["unique_id"]) == sorted(df["unique_id"])
        assert job.tables[0]["unique_id"].equals(table["unique_id"])
        l, r = job.pair_rows()
        rows.append(np.stack([l, r], axis=1))
        job.gammas(st)
        codes.append(job.gammas_host())
    exp = _pandas_block(table, [["surname"], ["dob"]])
    got_pairs = np.concatenate(rows)
    order = np.lexsort((got_pairs[:, 1], got_pairs[:, 0]))
    assert len(got_pairs) == len(exp)
    assert (got_pairs[order] == exp).all()
    gam = np.concatenate(codes)
    cols = [orc.StrCol(table[c].tolist()) for c in ["first_name", "surname", "dob", "city", "email"]]
    specs = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]
    ref = orc.template_gammas(specs, cols, cols, got_pairs[:, 0], got_pairs[:, 1])
    assert (gam == ref).all()


@pytest.mark.parametrize("link_type", ["dedupe_only", "link_only", "link_and_dedupe"])
def test_blocking_key_implied_levels(amd, link_type):
    """Pairs of a rule whose key includes the plain term `l.c = r.c` take column c's equal-strings
    level from the key (the filter reads no rows for them).  Against the oracle on every pair, with
    rules that must NOT imply equality next to ones that do: substr terms, an asymmetric term, a
    column holding the empty string, and a multi-term rule."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    df = _synthetic(6000, seed=17, surname_vocab=150, first_vocab=100, city_vocab=30)
    rng = np.random.Generator(np.random.PCG64(17))
    df.loc[rng.random(len(df)) < 0.05, "city"] = ""  # empty strings: city is never implied
    rules = ["l.surname = r.surname", "l.dob = r.dob and l.city = r.city",
             "substr(l.email, 1, 4) = substr(r.email, 1, 4)", "l.first_name = r.surname"]
    from splink_amd.synthetic import cfg_settings
    st = cfg_settings(2)  # first_name / surname JW-3, dob / city exact-2, email Lev-3
    st["link_type"] = link_type
    st["blocking_rules"] = rules
    st = complete_settings_dict(st, amd)
    inputs = [df] if link_type == "dedupe_only" else [df.iloc[:3000].reset_index(drop=True),
                                                       df.iloc[3000:].reset_index(drop=True)]
    if link_type == "link_and_dedupe":
        inputs = [pd.concat(inputs, ignore_index=True)]
        inputs[0]["_source_table"] = ["left"] * 3000 + ["right"] * 3000
    job = Job(link_type, inputs, "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    imp = job.ctx.gammas_implied_pairs(5)
    l, r = job.pair_rows()
    tl, tr = job.tables[0], job.r_table()
    cols = ["first_name", "surname", "dob", "city", "email"]
    specs = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]
    ref = orc.template_gammas(specs, [orc.StrCol(tl[c].tolist()) for c in cols],
                              [orc.StrCol(tr[c].tolist()) for c in cols], l, r)
    got = job.gammas_host()
    assert (got == ref).all(), np.nonzero((got != ref).any(axis=1))[0][:10]
    assert imp[1] > 0 and imp[2] > 0, imp       # surname (rule 0), dob (rule 1)
    assert imp[0] == 0 and imp[3] == 0 and imp[4] == 0, imp  # asymmetric, has "", substr
    # the interpreter path (no filter shortcut) agrees
    job.ctx.gammas_set_simple(0)
    job.gammas(st)
    assert (job.gammas_host() == ref).all()


def test_simple_columns_match_interpreter(amd):
    """The record-only filter for template-shaped columns and the general interpreter agree."""
    from splink_amd.engine import Job
    from splink_amd.synthetic import cfg_settings
    from splink_amd.settings import complete_settings_dict
    df = _synthetic(20000, seed=13, surname_vocab=500, first_vocab=300, city_vocab=80)
    df["dob_num"] = pd.to_numeric(df["dob"].str.replace("-", ""), errors="coerce")
    st = cfg_settings(2)
    from splink_amd import case_statements as cs
    extra = [("dob_abs4", cs.sql_gen_case_stmt_numeric_abs_4("dob_num", "dob_abs4", 1, 500), 4),
             ("dob_perc3", cs.sql_gen_case_stmt_numeric_perc_3("dob_num", "dob_perc3"), 3),
             ("dob_eq2", cs.sql_gen_case_stmt_numeric_2("dob_num", "dob_eq2"), 2),
             ("email4", cs.sql_gen_case_stmt_levenshtein_4("email", "email4"), 4),
             ("sn4", cs.sql_gen_gammas_case_stmt_jaro_4("surname", "sn4", 0.94, 0.88, 0.7), 4),
             ("fn2", cs.sql_gen_gammas_case_stmt_jaro_2("first_name", "fn2"), 2),
             ("city2", cs.sql_gen_case_smnt_strict_equality_2("city", "city2"), 2)]
    for name, expr, L in extra:
        st["comparison_columns"].append({"custom_name": name, "custom_columns_used": [name], "num_levels": L,
                                         "case_expression": expr})
    st = complete_settings_dict(st, amd)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    assert job.ctx.gammas_simple_count() == len(st["comparison_columns"])
    fast = job.gammas_host()
    job.ctx.gammas_set_simple(False)
    job.gammas(st)
    assert job.ctx.gammas_simple_count() == 0
    slow = job.gammas_host()
    assert (fast == slow).all()


@pytest.mark.parametrize("rules,big_rule1", [
    (["l.surname = r.surname", "l.dob = r.dob"], True),
    (["l.dob = r.dob", "l.first_name = r.first_name AND l.city = r.city", "l.surname = r.surname"], True),
    (["l.surname = r.surname", "l.first_name = r.surname"], False)])  # few rule-1 pairs: no whole view region
def test_rule_view_launch_matches_table_launch(amd, rules, big_rule1):
    """The second rule's pairs through its view-ordered image (forced, + 20) and through the table image
    (+ 10) give the oracle's comparison vectors -- symmetric, multi-term and asymmetric rules."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import cfg_settings
    df = _synthetic(12000, seed=29, surname_vocab=300, first_vocab=200, city_vocab=40)
    st = complete_settings_dict(cfg_settings(2), amd)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(rules)
    out = []
    for mode in (21, 11, 21):
        job.ctx.gammas_set_simple(mode)
        job.gammas(st)
        assert (job.ctx.gammas_view_regions() > 0) == (mode == 21 and big_rule1)
        out.append(job.gammas_host())
    assert (out[0] == out[1]).all() and (out[2] == out[1]).all()
    table = job.tables[0]
    l, r = job.pair_rows()
    cols = [orc.StrCol(table[c].tolist()) for c in ["first_name", "surname", "dob", "city", "email"]]
    specs = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]
    assert (out[0] == orc.template_gammas(specs, cols, cols, l, r)).all()


def test_em_at_scale_matches_oracle(amd):
    from splink_amd.engine import Job, m_step_rows
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings
    df = _synthetic(30000, seed=12, surname_vocab=600, first_vocab=400, city_vocab=100)
    settings = cfg_settings(2, max_iterations=10)
    params = Params(settings, amd)
    st = params.settings
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    gam = job.gammas_host()
    names, nlev = job.code_meta
    lam = params.params["λ"]
    lp = params._level_probabilities()
    hist_o, mp_o = orc.em_iterate(gam, nlev, lam, [m for m, _ in lp], [u for _, u in lp], 10, 1e-12)
    for lam_o, m_o, u_o in hist_o:
        stats = job.em_stats(params.params["λ"], params._level_probabilities())
        new_lambda, rows = m_step_rows(stats, names, nlev)
        params._update_params(new_lambda, rows)
        assert rel_close(params.params["λ"], lam_o)
        for k, (m, u) in enumerate(params._level_probabilities()):
            assert all(rel_close(a, b) for a, b in zip(m, m_o[k]))
            assert all(rel_close(a, b) for a, b in zip(u, u_o[k]))
    mp = job.score(params.params["λ"], params._level_probabilities())
    assert np.allclose(mp, mp_o, rtol=1e-9, atol=0)
    # ranges of the scoring kernel: odd / even start and length, single pairs, empty ranges
    lam = params.params["λ"]
    m_t, u_t = job.flat_tables(params._level_probabilities())
    n = len(mp)
    for start, count in [(0, 1), (1, 0), (1, 1), (1, 2), (1, 7), (2, 6), (3, n - 3), (n - 1, 1), (n - 2, 2)]:
        got = job.ctx.score(float(lam), float(1 - lam), m_t, u_t, start, count)
        assert np.array_equal(got, mp[start:start + count], equal_nan=True), (start, count)


def test_cross_column_equality(amd):
    """Dictionary ids are per column: `a_l = b_r` must compare strings, not ids of two spaces."""
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(5))
    vocab_a = ["x", "yy", "zzz", "shared", None]
    vocab_b = ["shared", "zzz", "q", None]
    n = 400
    pick = lambda v: rng.choice(np.array(v, dtype=object), n)  # noqa: E731
    df = pd.DataFrame({"a_l": pick(vocab_a), "a_r": pick(vocab_a), "b_l": pick(vocab_b), "b_r": pick(vocab_b)})
    expr = ("case when a_l is null or b_r is null then -1 when a_l = b_r then 2 "
            "when a_l = a_r then 1 else 0 end")
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "x", "custom_columns_used": ["a", "b"], "num_levels": 3, "case_expression": expr}]}
    got = add_gammas(df, st, amd).gamma_matrix()[:, 0]
    for k, (al, ar, br) in enumerate(zip(df.a_l, df.a_r, df.b_r)):
        if al is None or br is None:
            want = -1
        elif al == br:
            want = 2
        elif al == ar:
            want = 1
        else:
            want = 0
        assert got[k] == want, (al, br, ar)


def test_edge_cases(amd):
    from splink_amd import Splink
    # empty input: no pairs
    empty = pd.DataFrame({"unique_id": pd.Series([], dtype=np.int64), "name": pd.Series([], dtype=object)})
    st = {"link_type": "dedupe_only", "comparison_columns": [{"col_name": "name"}],
          "blocking_rules": ["l.name = r.name"], "max_iterations": 0}
    df_e = Splink(st, amd, df=empty).get_scored_comparisons()
    assert df_e.count() == 0 and len(df_e.toPandas()) == 0
    # every key NULL: no pairs; single record: no pairs
    df = pd.DataFrame({"unique_id": [1, 2, 3], "name": [None, None, None]})
    assert Splink(copy.deepcopy(st), amd, df=df).get_scored_comparisons().count() == 0
    # duplicate unique ids are never paired with each other
    df = pd.DataFrame({"unique_id": [1, 1, 2], "name": ["a", "a", "a"]})
    out = Splink(copy.deepcopy(st), amd, df=df).get_scored_comparisons().toPandas()
    assert sorted(zip(out.unique_id_l, out.unique_id_r)) == [(1, 2), (1, 2)]


@pytest.mark.parametrize("n_levels", [[2], [3, 3, 2, 2, 3], [4, 4, 4, 4, 4], [5, 5, 5, 5, 5, 5, 5], [4] * 9])
def test_em_histogram_kernels_agree(amd, n_levels):
    """Lane-private (R = 64 .. 4 copies) and wave-ballot histograms give the same pattern counts,
    from 3 to 2M patterns (uint16 and uint32 codes), skewed towards one dominant pattern."""
    from splink_amd import _native as N
    rng = np.random.Generator(np.random.PCG64(len(n_levels) * 7 + n_levels[0]))
    P = 1_000_003  # not a multiple of the 16-byte vector
    g = np.zeros((P, len(n_levels)), dtype=np.int8)
    for k, L in enumerate(n_levels):
        dominant = rng.random(P) < 0.8
        g[:, k] = np.where(dominant, 0, rng.integers(-1, L, P)).astype(np.int8)
    ctx = N.Context(0)
    ctx.gammas_load(n_levels, g)
    n_pat = ctx.n_patterns()
    stride = np.cumprod([1] + [L + 1 for L in n_levels[:-1]])
    codes = ((g.astype(np.int64) + 1) * stride).sum(axis=1)
    want = np.bincount(codes, minlength=n_pat)
    got = []
    for lanes in (1, 0, 2):  # 2: lane counters without the release fence before each last-arriver ticket
        ctx.em_set_lane_histogram(lanes)
        hist = np.zeros(n_pat, dtype=np.uint64)
        import torch
        d = torch.full((n_pat,), -1, dtype=torch.int64, device="cuda:0")
        torch.cuda.synchronize()  # torch's fill runs on its own stream
        ctx.em_histogram(d.data_ptr())  # zeroes the buffer itself
        hist[:] = d.cpu().numpy().astype(np.uint64)
        got.append(hist)
    assert (got[0] == want).all() and (got[1] == want).all() and (got[2] == want).all()
    # the one-launch E+M iteration (finalize in the last workgroup) with and without the fence: the same
    # statistics bit for bit
    lam, m, u = 0.3, [], []
    for L in n_levels:
        pm = np.linspace(1.0, 2.0, L)
        m += list(pm / pm.sum())
        u += list(pm[::-1] / pm.sum())
    n_stats = 5 + 4 * sum(L + 1 for L in n_levels)
    stats = []
    for mode in (1, 2):
        ctx.em_set_lane_histogram(mode)
        stats.append(ctx.em_iteration(lam, 1.0 - lam, m, u, n_stats))
    assert np.array_equal(stats[0], stats[1])
    # ... and equal to the per-pair oracle: with fewer than 64 lane copies (>= 641 patterns) k_em_iter counts
    # the most frequent pattern as P minus every other bin, so a stray or missing code would shift counts into
    # it; P is odd, past the last 16-byte vector
    ms, us, at = [], [], 0
    for L in n_levels:
        ms.append(m[at:at + L])
        us.append(u[at:at + L])
        at += L
    want = orc.em_stats(g, n_levels, lam, ms, us)
    got = stats[0]
    assert got[1] == want[1] == P and got[2] == want[2]
    assert np.allclose(got[[0]], want[[0]], rtol=1e-12, atol=0)
    assert np.array_equal(got[5::4], want[3::4]) and np.array_equal(got[6::4], want[4::4])  # counts
    assert np.allclose(got[7::4], want[5::4], rtol=1e-11, atol=1e-300)
    assert np.allclose(got[8::4], want[6::4], rtol=1e-11, atol=1e-300)


def _mutate(rng, s, k, alpha):
    s = list(s)
    for _ in range(k):
        op = int(rng.integers(3))
        i = int(rng.integers(len(s) + 1))
        if op == 0 or not s:
            s.insert(i, alpha[int(rng.integers(len(alpha)))])
        elif op == 1:
            del s[min(i, len(s) - 1)]
        else:
            s[min(i, len(s) - 1)] = alpha[int(rng.integers(len(alpha)))]
    return "".join(s)


def _lev_variants_agree(job, settings, want):
    """Every Levenshtein exact-pass kernel choice (spk_gammas_set_lev_kernel: one cell per lane, lane refill,
    refill in free-text columns only, the same without the character-bag decisions) gives the same codes."""
    try:
        for kern in (0, 1, 2, 3):
            job.ctx.gammas_set_lev_kernel(kern)
            job.gammas(settings)
            assert (job.gammas_host() == want).all(), kern
    finally:
        job.ctx.gammas_set_lev_kernel(2)


def test_levenshtein_levels_exact(amd):
    """Exact Levenshtein in the template exact pass (bit-plane path, unit path, the 128-bit plane path
    of the slow list and the global-memory pass): six `<=` levels reveal the distance up to 5, a
    ratio column checks the division; lengths straddle the 32-, 64- and 128-unit word sizes, with
    shared prefixes / suffixes, Latin-1 and supplementary-plane characters and NULLs."""
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(21))
    alpha = list("abcde") + ["é", "ü"]
    left, right = [], []
    for n in [0, 1, 2, 5, 17, 31, 32, 33, 40, 63, 64, 65, 80, 100, 116, 127, 128, 129]:
        for k in [0, 1, 2, 3, 5, 8]:
            for rep in range(6):
                a = "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), n))
                if rep == 4:
                    a = "prefix" + a + "suffix"
                b = _mutate(rng, a, k, alpha)
                if rep == 5 and n < 40:
                    b = b + "\U0001F600"  # surrogate pair: code points != units
                left.append(a)
                right.append(b)
    left += [None, "x", None]
    right += ["x", None, None]
    df = pd.DataFrame({"a_l": left, "a_r": right})
    exact = ("case when a_l is null or a_r is null then -1 "
             + " ".join(f"when levenshtein(a_l, a_r) <= {d} then {6 - d}" for d in range(6)) + " else 0 end")
    ratio = ("case when a_l is null or a_r is null then -1 when a_l = a_r then 3 "
             "when levenshtein(a_l, a_r)/((length(a_l) + length(a_r))/2) <= 0.2 then 2 "
             "when levenshtein(a_l, a_r)/((length(a_l) + length(a_r))/2) <= 0.4 then 1 else 0 end")
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "lv", "custom_columns_used": ["a"], "num_levels": 7, "case_expression": exact,
         "m_probabilities": [0.1, 0.1, 0.1, 0.1, 0.1, 0.2, 0.3], "u_probabilities": [0.4, 0.2, 0.1, 0.1, 0.1, 0.05, 0.05]},
        {"custom_name": "lr", "custom_columns_used": ["a"], "num_levels": 4, "case_expression": ratio}]}
    gf = add_gammas(df, st, amd)
    got = gf.gamma_matrix()
    for i, (a, b) in enumerate(zip(left, right)):
        if a is None or b is None:
            assert got[i, 0] == -1 and got[i, 1] == -1
            continue
        d = orc.levenshtein(a, b)
        assert got[i, 0] == (6 - d if d <= 5 else 0), (a, b, d, got[i, 0])
        if a == b:
            want = 3
        else:
            den = (len(a) + len(b)) / 2.0
            q = d / den if den else None
            want = 2 if q is not None and q <= 0.2 else (1 if q is not None and q <= 0.4 else 0)
        assert got[i, 1] == want, (a, b, d, got[i, 1])
    _lev_variants_agree(gf.job, gf.settings, got)


@pytest.mark.parametrize("alpha,planes", [
    (list("0123456789-"), 5),          # bits 7, 6, 5 the same for every unit: 5 planes
    (list("abcdefghijklmnopqrstuvwxyz"), 5),
    (list("abcxyz.@_-0123"), 7),       # ASCII: plane 7 dropped
    (list("abcde") + ["é", "ü"], 8)])  # Latin-1: all 8 planes
def test_levenshtein_reduced_planes(amd, alpha, planes):
    """Levenshtein template levels when the scans skip the top bit-planes a column's units all share
    (SimpleCol.np): distances up to 5 and the ratio levels against the oracle, rows of 0-128 units
    (one- and two-word planes), shared prefixes / suffixes and NULLs."""
    from splink_amd import case_statements as cs
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(len(alpha)))
    left, right = [], []
    for n in [0, 1, 3, 12, 31, 32, 33, 47, 64, 65, 90, 128]:
        for k in [0, 1, 2, 4, 7]:
            for rep in range(4):
                a = "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), n))
                b = _mutate(rng, a, k, alpha)[:128]
                if rep == 3:
                    b = "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), len(b)))
                left.append(a)
                right.append(b)
    left += [None, alpha[0]]
    right += [alpha[0], None]
    df = pd.DataFrame({"a_l": left, "a_r": right})
    exact = ("case when a_l is null or a_r is null then -1 "
             + " ".join(f"when levenshtein(a_l, a_r) <= {d} then {6 - d}" for d in range(6)) + " else 0 end")
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "lv", "custom_columns_used": ["a"], "num_levels": 7, "case_expression": exact,
         "m_probabilities": [0.1, 0.1, 0.1, 0.1, 0.1, 0.2, 0.3], "u_probabilities": [0.4, 0.2, 0.1, 0.1, 0.1, 0.05, 0.05]},
        {"custom_name": "lr", "custom_columns_used": ["a"], "num_levels": 4,
         "case_expression": cs.sql_gen_case_stmt_levenshtein_4("a")}]}
    gf = add_gammas(df, st, amd)
    got = gf.gamma_matrix()
    for i, (a, b) in enumerate(zip(left, right)):
        if a is None or b is None:
            assert got[i, 0] == -1 and got[i, 1] == -1
            continue
        d = orc.levenshtein(a, b)
        assert got[i, 0] == (6 - d if d <= 5 else 0), (a, b, d, got[i, 0])
        den = (len(a) + len(b)) / 2.0
        want = 3 if a == b else (2 if den and d / den <= 0.2 else (1 if den and d / den <= 0.4 else 0))
        assert got[i, 1] == want, (a, b, d, got[i, 1])
    _lev_variants_agree(gf.job, gf.settings, got)


def test_exact_work_lists_grow(amd):
    """More undecided cells than the exact-pass lists hold on the first try (3 columns x 40k pairs of
    anagrams, which no length / letter-count bound decides): the lists are re-sized on the device
    side and the pass re-run, with the same levels as the oracle."""
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(33))
    n = 40000
    base = np.array(list("abcdefghij"))
    data = {}
    for c in ("x", "y", "z"):
        data[f"{c}_l"] = ["".join(rng.permutation(base)) for _ in range(n)]
        data[f"{c}_r"] = ["".join(rng.permutation(base)) for _ in range(n)]
    df = pd.DataFrame(data)
    expr = ("case when {c}_l is null or {c}_r is null then -1 when levenshtein({c}_l, {c}_r) <= 5 then 2 "
            "when levenshtein({c}_l, {c}_r) <= 7 then 1 else 0 end")
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": c, "custom_columns_used": [c], "num_levels": 3, "case_expression": expr.format(c=c)}
        for c in ("x", "y", "z")]}
    got = add_gammas(df, st, amd).gamma_matrix()
    for j, c in enumerate(("x", "y", "z")):
        d = np.array([orc.levenshtein(a, b) for a, b in zip(data[f"{c}_l"], data[f"{c}_r"])])
        want = np.where(d <= 5, 2, np.where(d <= 7, 1, 0))
        assert (got[:, j] == want).all(), c


def test_cfg5_address_column_at_scale(amd):
    """cfg5's columns: blocking surname|dob over records with 30-128 character free-text addresses
    (Levenshtein-4, case_statements.py:128-141) next to the five cfg2 columns -- pair set and every
    gamma against the C oracle; most address cells are decided by the 128-bit plane path."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import cfg_settings, make_records
    cols = ["first_name", "surname", "dob", "city", "email", "address"]
    df = make_records(20000, seed=17, surname_vocab=400, first_vocab=300, city_vocab=60,
                      with_address=True)[["unique_id"] + cols]
    assert (df["address"].dropna().str.len() > 64).mean() > 0.2
    st = complete_settings_dict(cfg_settings(5), amd)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    table = job.tables[0]
    l, r = job.pair_rows()
    exp = _pandas_block(table, [["surname"], ["dob"]])
    got_pairs = np.stack([l, r], axis=1)
    order = np.lexsort((got_pairs[:, 1], got_pairs[:, 0]))
    assert (got_pairs[order] == exp).all()
    job.gammas(st)
    gam = job.gammas_host()
    ocols = [orc.StrCol(table[c].tolist()) for c in cols]
    specs = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3]),
             ("lev", 4, [0.2, 0.4])]
    ref = orc.template_gammas(specs, ocols, ocols, l, r)
    assert (gam == ref).all()
    assert len(np.unique(gam[:, 5])) == 5  # every address level occurs
    # the slow-list kernels (65-128-unit addresses) left to the settlement at the next synchronising call,
    # as happens when the previous call with the same inputs had empty slow lists: same comparison vectors
    assert job.ctx.gammas_deferred() > 0
    job.ctx.gammas_set_simple(101)
    for _ in range(2):
        job.gammas(st)
        assert (job.gammas_host() == ref).all()
    job.ctx.gammas_set_simple(1)
    job.gammas(st)
    assert (job.gammas_host() == ref).all()
    # every Levenshtein exact-pass kernel (one cell per lane, lane refill, auto): the same vectors
    _lev_variants_agree(job, st, ref)


def test_row_image_rebuilt_when_layout_changes(amd):
    """The filter's row image is kept across comparison passes of one context and rebuilt when the
    simple-column layout or a table changes: alternating settings give the same codes every time."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import cfg_settings
    df = _synthetic(8000, seed=19, surname_vocab=300, first_vocab=200, city_vocab=50)
    st = complete_settings_dict(cfg_settings(2), amd)
    st2 = copy.deepcopy(cfg_settings(2))
    st2["comparison_columns"] = [st2["comparison_columns"][i] for i in (4, 0, 3)]  # email, first_name, city
    st2 = complete_settings_dict(st2, amd)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    g1 = job.gammas_host()
    job.gammas(st2)
    h1 = job.gammas_host()
    assert (h1 == g1[:, [4, 0, 3]]).all()
    job.gammas(st)
    assert (job.gammas_host() == g1).all()
    job.gammas(st2)
    assert (job.gammas_host() == h1).all()


def _two_ranks(tmp_path, mode=None):
    """Run tests/gpu_dist_worker.py as two gloo ranks on cuda:0; returns their JSON outputs."""
    import json
    import os
    import socket
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "rank")
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LOCAL_RANK="0")
        cmd = [sys.executable, os.path.join(here, "gpu_dist_worker.py"), out] + ([mode] if mode else [])
        procs.append(subprocess.Popen(cmd, env=env))
    for p in procs:
        assert p.wait(timeout=170) == 0
    return [json.load(open(f"{out}.{r}")) for r in range(2)]


def test_sharded_ranks_match_oracle(amd, tmp_path):
    """Two ranks (child processes, gloo, both on cuda:0) run the sharded device path -- pair-ordinal
    shards of spk_block, per-rank comparison vectors, histogram all-reduce per EM iteration -- and
    end with the oracle's parameters (C restatement over all pairs, at 1e-9), and bit for bit with
    one process over all pairs."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import gpu_dist_worker as W
    ranks = _two_ranks(tmp_path)
    single, job, (lam0, lp0), nlev = W.run((0, 1), want_job=True)
    assert ranks[0]["n_pairs"] > 0 and ranks[1]["n_pairs"] > 0
    assert ranks[0]["n_pairs"] + ranks[1]["n_pairs"] == single["n_pairs"]
    # the oracle over every pair, independent of the device's comparison vectors and EM
    l, r = job.pair_rows()
    table = job.tables[0]
    cols = [orc.StrCol(table[c].tolist()) for c in W.COLS]
    specs = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]
    gam = orc.template_gammas(specs, cols, cols, l, r)
    hist_o, _ = orc.em_iterate(gam, nlev, lam0, [m for m, _ in lp0], [u for _, u in lp0], W.ITERS, 1e-300)
    lam_o, m_o, u_o = hist_o[-1]
    for rk in ranks:
        assert rel_close(rk["lambda"], lam_o)
        for k, (m, u) in enumerate(rk["pi"]):
            assert all(rel_close(a, b) for a, b in zip(m, m_o[k])), (k, m, m_o[k])
            assert all(rel_close(a, b) for a, b in zip(u, u_o[k]))
        assert rk["lambda"] == single["lambda"] and rk["pi"] == single["pi"]
        # each rank uploaded half of every string column and gathered the rest from the other rank: its
        # encoded table is byte-identical to the single process's local ingest
        assert rk["replicated_ingest"] and not single["replicated_ingest"]
        assert rk["table_digest"] == single["table_digest"]


def test_sharded_link_tf_matches_reference(amd, tmp_path):
    """link_only with term-frequency adjustment on two gloo ranks on cuda:0: each rank scores its
    shard of the pairs; the EM histogram and the per-value tf (Σmp, count) tables are all-reduced
    (term_frequencies.py:49-65 groups over all pairs).  The ranks' frames together are the golden."""
    g = load_golden("link_tf")
    ranks = _two_ranks(tmp_path, "link_tf")
    assert all(rk["n_pairs"] > 0 for rk in ranks)
    assert ranks[0]["lambda"] == ranks[1]["lambda"]
    for key in ("df_e", "df_tf"):
        cols = ranks[0][f"{key}_columns"]
        both = pd.concat([pd.DataFrame(rk[key])[cols] for rk in ranks], ignore_index=True)
        compare_frames(both, g[key], g[f"{key}_columns"])


def test_tf_bit_identical_across_runs_and_ranks(amd, tmp_path):
    """term_frequencies.py:49-65 sums mp per value over all pairs.  The device sums are exact fixed-point
    accumulators (integer adds in any order, all-reduced as integers), so tf_adjusted_match_prob is bit
    for bit the same in repeated runs and whether the pairs sit on one rank or are sharded over two."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import gpu_dist_worker as W
    one = W.run_link_tf()
    again = W.run_link_tf()
    assert one["df_tf"]["tf_adjusted_match_prob"] == again["df_tf"]["tf_adjusted_match_prob"]
    ranks = _two_ranks(tmp_path, "link_tf")
    cols = one["df_tf_columns"]
    both = pd.concat([pd.DataFrame(rk["df_tf"])[cols] for rk in ranks], ignore_index=True)
    single = pd.DataFrame(one["df_tf"])[cols]
    key = ["unique_id_l", "unique_id_r"]
    both = both.sort_values(key).reset_index(drop=True)
    single = single.sort_values(key).reset_index(drop=True)
    assert both[key].equals(single[key])
    a = both["tf_adjusted_match_prob"].to_numpy(dtype=np.float64)
    b = single["tf_adjusted_match_prob"].to_numpy(dtype=np.float64)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("P", [1, 7, 8, 9, 4097, 131075])
def test_em_first_launch_small_pair_sets(amd, P):
    """The first E+M launch on a pair set guesses its uncounted pattern from a sample (k_em_hot_sample; below
    one 16-byte vector of codes it counts them all): exact counts for pair sets around the vector width, in a
    3125-pattern space (8 lane copies), on fresh contexts so every launch here is a first one."""
    import torch
    from splink_amd import _native as N
    n_levels = [4] * 5
    rng = np.random.Generator(np.random.PCG64(P))
    g = rng.integers(-1, 4, (P, 5)).astype(np.int8)
    g[: P // 2] = 2  # one pattern holds half of the pairs
    stride = np.cumprod([1] + [L + 1 for L in n_levels[:-1]])
    want = np.bincount(((g.astype(np.int64) + 1) * stride).sum(axis=1), minlength=5 ** 5)
    for first in ("histogram", "iteration"):
        ctx = N.Context(0)
        ctx.gammas_load(n_levels, g)
        if first == "iteration":
            m = [0.25] * 20
            stats = ctx.em_iteration(0.3, 0.7, m, m, 5 + 4 * 25)
            assert stats[1] == P
        d = torch.full((5 ** 5,), -1, dtype=torch.int64, device="cuda:0")
        torch.cuda.synchronize()
        ctx.em_histogram(d.data_ptr())
        assert np.array_equal(d.cpu().numpy(), want)


def test_levenshtein_bag_decisions(amd):
    """Character-bag decisions before the free-text exact pass (k_bag_rows / k_compact_lev): address-like
    strings of 20-140 units (mixed case, digits, spaces, punctuation, Latin-1 and supplementary-plane
    characters, NULLs), unrelated pairs (mostly decided by their bags) and near copies (scanned); levels equal
    the oracle's, some list slots were decided (-1), and every kernel mode, with and without the decisions,
    gives the same codes.  Buckets saturate on long runs of one letter, which the bound then leaves alone."""
    from splink_amd.gammas import add_gammas
    rng = np.random.Generator(np.random.PCG64(77))
    alpha = list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 ,.-()") + ["é", "ß", "\U0001F600"]
    def rnd(n):
        return "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), n))
    left, right = [], []
    for n in [20, 40, 63, 64, 65, 66, 90, 127, 128, 140]:
        for rep in range(40):
            a = rnd(n)
            if rep < 25:
                b = rnd(int(rng.integers(max(1, n - 10), n + 10)))  # unrelated
            elif rep < 35:
                b = _mutate(rng, a, int(rng.integers(0, max(2, n // 4))), alpha[:62])  # near copy
            elif rep < 38:
                a = "a" * n
                b = "a" * (n - 3) + "bcd"  # a bucket saturated on both sides
            else:
                b = a
            left.append(a)
            right.append(b)
    left += [None, "x" * 70, None]
    right += ["y" * 70, None, None]
    df = pd.DataFrame({"a_l": left, "a_r": right})
    ratio = ("case when a_l is null or a_r is null then -1 when a_l = a_r then 3 "
             "when levenshtein(a_l, a_r)/((length(a_l) + length(a_r))/2) <= 0.2 then 2 "
             "when levenshtein(a_l, a_r)/((length(a_l) + length(a_r))/2) <= 0.4 then 1 else 0 end")
    st = {"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": "lr", "custom_columns_used": ["a"], "num_levels": 4, "case_expression": ratio}]}
    gf = add_gammas(df, st, amd)
    got = gf.gamma_matrix()
    for i, (a, b) in enumerate(zip(left, right)):
        if a is None or b is None:
            assert got[i, 0] == -1
            continue
        if a == b:
            assert got[i, 0] == 3
            continue
        d = orc.levenshtein(a, b)
        ca, cb = len(a.encode("utf-16-le")) // 2, len(b.encode("utf-16-le")) // 2
        q = d / ((len(a) + len(b)) / 2.0)
        want = 2 if q <= 0.2 else (1 if q <= 0.4 else 0)
        assert got[i, 0] == want, (a, b, d, ca, cb, got[i, 0])
    n_exact = gf.job.ctx.gammas_exact_counts(1)[0]
    items = gf.job.ctx.gammas_exact_list(0, int(n_exact))
    assert (items < 0).sum() > 0, "no cell was decided from its character bag"
    _lev_variants_agree(gf.job, gf.settings, got)
