"""Generate golden parity fixtures from the REFERENCE implementation (run in the build container only).

The reference (splink 0.1.7 at /root/reference) is pure Python that emits Spark
SQL.  pyspark and the JVM are absent, so this script drives the reference's own
SQL generators (`_sql_gen_*`) and its `Params` / `complete_settings_dict`
through sqlite3, patched to Spark semantics where sqlite differs (SURVEY.md §7,
§8(c)):

* `jaro_winkler_sim` -- registered UDF, a pure-Python restatement of the
  commons-text 1.4 bytecode spec on UTF-16 code units;
* `levenshtein` / `length` -- registered to return doubles, so the Levenshtein
  template divides in double exactly like Spark (sqlite would integer-divide);
* `cast(... as float)` in the M-step -- sqlite keeps double, so the λ / π
  values are rounded to IEEE binary32 here, as Spark does;
* the EM loop follows splink/iterate.py:37-63 exactly, calling the reference
  `Params._update_params` and `Params.is_converged`.

Outputs are written as JSON fixtures next to this script.  Nothing here is
imported by the product, and the reference never travels to the GPU box.

Usage:  PYTHONPATH=/root/reference python tests/golden/make_golden.py
"""
from __future__ import annotations

import copy
import json
import math
import os
import sqlite3
import sys
import warnings

import numpy as np
import pandas as pd

warnings.filterwarnings("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("SPLINK_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from splink.blocking import (  # noqa: E402  (reference)
    _get_columns_to_retain_blocking, _sql_gen_block_using_rules, _sql_gen_cartesian_block,
    _sql_gen_vertically_concatenate)
from splink.case_statements import (  # noqa: E402
    sql_gen_case_smnt_strict_equality_2, sql_gen_case_stmt_levenshtein_3, sql_gen_case_stmt_levenshtein_4,
    sql_gen_case_stmt_numeric_abs_3, sql_gen_case_stmt_numeric_abs_4, sql_gen_case_stmt_numeric_perc_3,
    sql_gen_case_stmt_numeric_perc_4, sql_gen_gammas_case_stmt_jaro_2, sql_gen_gammas_case_stmt_jaro_3,
    sql_gen_gammas_case_stmt_jaro_4, sql_gen_gammas_name_inversion_4, sql_gen_case_stmt_numeric_2)
from splink.expectation_step import (  # noqa: E402
    _sql_gen_expected_match_prob, _sql_gen_gamma_prob_columns, get_overall_log_likelihood)
from splink.gammas import _sql_gen_add_gammas  # noqa: E402
from splink.maximisation_step import (  # noqa: E402
    _sql_gen_intermediate_pi_aggregate, _sql_gen_new_lambda, _sql_gen_pi_df)
from splink.params import Params  # noqa: E402
from splink.settings import complete_settings_dict  # noqa: E402
from splink.term_frequencies import (  # noqa: E402
    sql_gen_add_adjumentments_to_df_e, sql_gen_compute_final_group_membership_prob_from_adjustments,
    sql_gen_generate_adjusted_lambda)

from splink_amd.synthetic import make_records, CONFIGS, cfg_settings  # noqa: E402


# --------------------------------------------------------------------------------------
# Spark-semantics UDFs (independent pure-Python restatements used only for the goldens)
# --------------------------------------------------------------------------------------
def _u16(s: str):
    b = s.encode("utf-16-le", "surrogatepass")
    return [b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2)]


def py_jaro_winkler(a, b):
    """commons-text 1.4 JaroWinklerDistance.apply, UTF-16 code units."""
    if a is None or b is None:
        return None
    first, second = _u16(a), _u16(b)
    if len(first) > len(second):
        mx, mn = first, second
    else:
        mx, mn = second, first
    rng = max(len(mx) // 2 - 1, 0)
    idx = [-1] * len(mn)
    flags = [False] * len(mx)
    m = 0
    for mi, c in enumerate(mn):
        for xi in range(max(mi - rng, 0), min(mi + rng + 1, len(mx))):
            if not flags[xi] and c == mx[xi]:
                idx[mi] = xi
                flags[xi] = True
                m += 1
                break
    ms1 = [mn[i] for i in range(len(mn)) if idx[i] != -1]
    ms2 = [mx[i] for i in range(len(mx)) if flags[i]]
    trans = sum(1 for x, y in zip(ms1, ms2) if x != y)
    prefix = 0
    for mi in range(len(mn)):
        if first[mi] == second[mi]:
            prefix += 1
        else:
            break
    if m == 0:
        return 0.0
    md = float(m)
    j = ((md / len(first) + md / len(second)) + (md - float(trans // 2)) / md) / 3.0
    if j < 0.7:
        return j
    return j + (min(0.1, 1.0 / len(mx)) * prefix) * (1.0 - j)


def py_levenshtein(a, b):
    """Spark UTF8String.levenshteinDistance: unit-cost edit distance over code points."""
    if a is None or b is None:
        return None
    s, t = list(a), list(b)
    prev = list(range(len(t) + 1))
    for i, cs in enumerate(s, 1):
        cur = [i] + [0] * len(t)
        for j, ct in enumerate(t, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (cs != ct))
        prev = cur
    return float(prev[-1])


def py_length(a):
    return None if a is None else float(len(a))


def f32(x):
    return None if x is None else float(np.float32(x))


def spark_ln(x):
    """Spark's ln: NULL for x <= 0 (and for NULL)."""
    return None if x is None or x <= 0 else math.log(x)


def connect():
    con = sqlite3.connect(":memory:")
    con.row_factory = sqlite3.Row
    con.create_function("ln", 1, spark_ln, deterministic=True)
    con.create_function("jaro_winkler_sim", 2, py_jaro_winkler, deterministic=True)
    con.create_function("levenshtein", 2, py_levenshtein, deterministic=True)
    con.create_function("length", 1, py_length, deterministic=True)
    return con


class _Fn:
    name = "jaro_winkler_sim"


class JaroSpark:
    """Stand-in for a SparkSession on which the jar's UDF is registered (case_statements.py:12-14)."""

    class catalog:  # noqa: N801
        @staticmethod
        def listFunctions():
            return [_Fn()]


class SqliteFrame:
    """The slice of a Spark DataFrame that the reference's get_overall_log_likelihood touches
    (expectation_step.py:224-272): createOrReplaceTempView, groupby().sum(col).collect()."""

    def __init__(self, con, sql):
        self.con, self.sql = con, sql
        self._agg = None

    def createOrReplaceTempView(self, name):  # noqa: N802
        self.con.execute(f"drop view if exists {name}")
        self.con.execute(f"create temp view {name} as {self.sql}")

    def groupby(self):
        return self

    def sum(self, col):
        out = SqliteFrame(self.con, self.sql)
        out._agg = col
        return out

    def collect(self):
        return [[self.con.execute(f"select sum({self._agg}) from ({self.sql})").fetchone()[0]]]


class SqliteSpark:
    """spark.sql over the sqlite connection (lazy, like Spark)."""

    def __init__(self, con):
        self.con = con

    def sql(self, sql):
        return SqliteFrame(self.con, sql)


def spark_for(jaro):
    return JaroSpark() if jaro else "supress_warnings"


def q(con, sql):
    return pd.read_sql(sql, con)


def to_table(con, df, name):
    df.to_sql(name, con, index=False)


def jsonable(v):
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating, float)):
        v = float(v)
        return None if math.isnan(v) else v
    if isinstance(v, (np.bool_,)):
        return bool(v)
    return v


def frame_json(df):
    return {c: [jsonable(v) for v in df[c].tolist()] for c in df.columns}


def sort_pairs(df):
    keys = [k for k in ("_source_table_l", "unique_id_l", "_source_table_r", "unique_id_r") if k in df.columns]
    rest = [c for c in df.columns if c.startswith("gamma_")]
    return df.sort_values(keys + rest, kind="mergesort").reset_index(drop=True)


def params_snapshot(params):
    p = params.params
    out = {"lambda": p["λ"], "pi": {}}
    for g, d in p["π"].items():
        out["pi"][g] = {
            "m": [d["prob_dist_match"][f"level_{i}"]["probability"] for i in range(d["num_levels"])],
            "u": [d["prob_dist_non_match"][f"level_{i}"]["probability"] for i in range(d["num_levels"])],
        }
    return out


# --------------------------------------------------------------------------------------
# Reference pipeline: block -> gammas -> EM (iterate.py semantics) -> final E (-> tf)
# --------------------------------------------------------------------------------------
def reference_pipeline(settings_in, jaro, df=None, df_l=None, df_r=None, df_gammas=None, tf=False, ll=False):
    spark = spark_for(jaro)
    settings = complete_settings_dict(copy.deepcopy(settings_in), spark)
    con = connect()
    link_type = settings["link_type"]
    uid = settings["unique_id_column_name"]
    out = {"settings_in": settings_in, "jaro": jaro, "link_type": link_type}

    if df_gammas is None:
        if df is not None:
            out["df"] = frame_json(df)
        if df_l is not None:
            out["df_l"] = frame_json(df_l)
            out["df_r"] = frame_json(df_r)
        cols = _get_columns_to_retain_blocking(settings)
        if link_type == "dedupe_only":
            to_table(con, df, "df")
        elif link_type == "link_only":
            to_table(con, df_l, "df_l")
            to_table(con, df_r, "df_r")
        else:
            to_table(con, df_l, "df_l")
            to_table(con, df_r, "df_r")
            con.execute(f"create table df as {_sql_gen_vertically_concatenate(list(cols))}")
            cols = cols + ["_source_table"]
        rules = settings.get("blocking_rules", [])
        if rules:
            sql = _sql_gen_block_using_rules(link_type, list(cols), rules, uid)
        else:
            sql = _sql_gen_cartesian_block(link_type, list(cols), uid)
        con.execute(f"create table df_comparison as {sql}")
        con.execute("create table df_gammas as " + _sql_gen_add_gammas(settings, uid, "df_comparison"))
        g = sort_pairs(q(con, "select * from df_gammas"))
        out["gammas"] = frame_json(g)
    else:
        to_table(con, df_gammas, "df_gammas")
        out["df_gammas"] = frame_json(df_gammas)

    params = Params(settings, spark)
    out["settings_completed"] = params.settings
    out["initial"] = params_snapshot(params)
    try:
        _em(con, params, settings, out, tf, ll)
    except Exception as e:  # the reference itself fails here; record the error it raises
        out["error"] = type(e).__name__
    return out


def _log_likelihood(con, params):
    """The reference's own get_overall_log_likelihood (expectation_step.py:259-272) on df_wgp."""
    return get_overall_log_likelihood(SqliteFrame(con, "select * from df_wgp"), params, SqliteSpark(con))


def _em(con, params, settings, out, tf, ll=False):
    iters = []
    out["iterations"] = iters
    lls = []
    if ll:
        out["log_likelihood"] = lls  # one per E-step (iterate.py:45-63 with compute_ll=True)
    for _ in range(settings["max_iterations"]):
        con.execute("drop table if exists df_wgp")
        con.execute("drop table if exists df_e")
        con.execute("drop table if exists df_intermediate")
        con.execute("create table df_wgp as " + _sql_gen_gamma_prob_columns(params, settings, "df_gammas"))
        if ll:
            lls.append(_log_likelihood(con, params))
        con.execute("create table df_e as " + _sql_gen_expected_match_prob(params, settings, "df_wgp"))
        con.execute("create table df_intermediate as " + _sql_gen_intermediate_pi_aggregate(params, "df_e"))
        new_lambda = f32(con.execute(_sql_gen_new_lambda("df_intermediate")).fetchone()[0])
        rows = [dict(r) for r in con.execute(_sql_gen_pi_df(params, "df_intermediate")).fetchall()]
        for r in rows:
            r["new_probability_match"] = f32(r["new_probability_match"])
            r["new_probability_non_match"] = f32(r["new_probability_non_match"])
        params._update_params(new_lambda, rows)
        snap = params_snapshot(params)
        snap["pi_rows"] = rows
        iters.append(snap)
        if params.is_converged():
            break
    out["final_iteration"] = params.iteration
    con.execute("drop table if exists df_wgp")
    con.execute("drop table if exists df_e")
    con.execute("create table df_wgp as " + _sql_gen_gamma_prob_columns(params, settings, "df_gammas"))
    if ll:
        lls.append(_log_likelihood(con, params))
    con.execute("create table df_e as " + _sql_gen_expected_match_prob(params, settings, "df_wgp"))
    df_e = q(con, "select * from df_e")
    out["df_e_columns"] = list(df_e.columns)
    out["df_e"] = frame_json(sort_pairs(df_e))

    if tf:
        tf_cols = [c["col_name"] for c in settings["comparison_columns"] if c["term_frequency_adjustments"]]
        for c in tf_cols:
            con.execute(f"create table {c}_lookup as " + sql_gen_generate_adjusted_lambda(c, params, "df_e"))
        con.execute("create table df_e_adj as " + sql_gen_add_adjumentments_to_df_e(tf_cols))
        sql = sql_gen_compute_final_group_membership_prob_from_adjustments(tf_cols, settings, "df_e_adj")
        df_tf = q(con, sql)
        out["df_tf_columns"] = list(df_tf.columns)
        out["df_tf"] = frame_json(sort_pairs(df_tf))


def dump(name, obj):
    path = os.path.join(HERE, f"{name}.json")
    with open(path, "w") as f:
        json.dump(obj, f, ensure_ascii=False, separators=(",", ":"))
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


# --------------------------------------------------------------------------------------
# Datasets (tests/conftest.py fixtures of the reference, restated as data)
# --------------------------------------------------------------------------------------
def test1_records():  # reference tests/conftest.py:147-154
    return pd.DataFrame({
        "unique_id": [1, 2, 3, 4, 5, 6, 7],
        "mob": [10, 10, 10, 7, 8, 8, 8],
        "surname": ["Linacre", "Linacre", "Linacer", "Smith", "Smith", "Smith", "Jones"]})


SUBSTR_CASE = """
            case
            when surname_l is null or surname_r is null then -1
            when surname_l = surname_r then 2
            when substr(surname_l,1, 3) =  substr(surname_r, 1, 3) then 1
            else 0
            end
            as gamma_surname
            """


def gamma_settings_1():  # reference tests/conftest.py:98-126
    return {
        "link_type": "dedupe_only", "proportion_of_matches": 0.4,
        "comparison_columns": [
            {"col_name": "mob", "num_levels": 2, "m_probabilities": [0.1, 0.9], "u_probabilities": [0.8, 0.2]},
            {"col_name": "surname", "num_levels": 3, "case_expression": SUBSTR_CASE,
             "m_probabilities": [0.1, 0.2, 0.7], "u_probabilities": [0.5, 0.25, 0.25]}],
        "blocking_rules": ["l.mob = r.mob", "l.surname = r.surname"],
        "max_iterations": 2,
    }


def gamma_settings_2():  # reference tests/conftest.py:246-283
    return {
        "link_type": "dedupe_only", "proportion_of_matches": 0.1,
        "comparison_columns": [
            {"col_name": "forename", "num_levels": 2, "m_probabilities": [0.4, 0.6], "u_probabilities": [0.65, 0.35]},
            {"col_name": "surname", "num_levels": 3, "case_expression": SUBSTR_CASE,
             "m_probabilities": [0.05, 0.2, 0.75], "u_probabilities": [0.4, 0.3, 0.3]},
            {"col_name": "dob", "num_levels": 2, "m_probabilities": [0.4, 0.6], "u_probabilities": [0.65, 0.35]}],
        "blocking_rules": [],
        "max_iterations": 3,
    }


def test2_records():  # reference tests/conftest.py:303-309
    return pd.DataFrame({
        "unique_id": [1, 2, 3, 4],
        "forename": ["Robin", "Robin", "Robin", None],
        "surname": ["Linacre", "Linacre", None, None],
        "dob": ["1980-01-01", None, None, None]})


def dgp_gammas():  # reference tests/conftest.py:418-473 (known data-generating process)
    cols = ["col_2_levels", "col_5_levels", "col_20_levels"]

    def build(probs, agree_first):
        df = None
        for i, p in enumerate(probs):
            n = int(1 / p)
            vals = ([0] * (n - 1) + [1]) if agree_first else ([1] * (n - 1) + [0])
            d = pd.DataFrame({f"gamma_{cols[i]}": vals, "join_col": [1] * n})
            df = d if df is None else df.merge(d, on="join_col")
        return df.drop("join_col", axis=1)

    nm = build([0.05, 0.2, 0.5], True)
    m = build([0.05, 0.1, 0.05], False)
    df = pd.concat([nm, m]).reset_index(drop=True).reset_index().rename(columns={"index": "unique_id_l"})
    df["unique_id_r"] = df["unique_id_l"]
    return df[["unique_id_l", "unique_id_r"] + [f"gamma_{c}" for c in cols]]


def gamma_settings_4():
    return {
        "link_type": "dedupe_only", "proportion_of_matches": 0.9,
        "comparison_columns": [
            {"col_name": c, "num_levels": 2, "case_expression": sql_gen_case_smnt_strict_equality_2(c)}
            for c in ["col_2_levels", "col_5_levels", "col_20_levels"]],
        "blocking_rules": [], "retain_matching_columns": False,
        "em_convergence": 0.001, "max_iterations": 40,
    }


def link_data(repeat_ids):  # reference tests/conftest.py:36-94
    if repeat_ids:
        l = pd.DataFrame({"unique_id": [1, 2, 3], "surname": ["Linacre", "Smith", "Smith"],
                          "first_name": ["Robin", "John", "John"]})
        r = pd.DataFrame({"unique_id": [1, 2, 3], "surname": ["Linacre", "Smith", "Smith"],
                          "first_name": ["Robin", "John", "Robin"]})
    else:
        l = pd.DataFrame({"unique_id": [1, 2], "surname": ["Linacre", "Smith"], "first_name": ["Robin", "John"]})
        r = pd.DataFrame({"unique_id": [7, 8, 9], "surname": ["Linacre", "Smith", "Smith"],
                          "first_name": ["Robin", "John", "Robin"]})
    return l, r


def blocks_records():  # reference tests/test_blocks.py:13-19
    return pd.DataFrame({"unique_id": [1, 2, 3, 4, 5, 6],
                         "first_name": ["robin", "john", "john", "john", None, "john"],
                         "surname": ["linacre", "smith", "linacre", "smith", "smith", None]})


def case_level_tables():
    """Reference tests/test_case_statements.py + tests/test_spark.py:314-419 inputs, every template."""
    con = connect()
    strs = pd.DataFrame({
        "str_col_l": ["these strings are equal", "these strings are almost equal", "these strings are almost equal",
                      "these strings are almost equal", None, "", "", "smith", "Ünïcødé", "a\U0001F600b", "MARTHA",
                      "DWAYNE", "DIXON", "abc", "x"],
        "str_col_r": ["these strings are equal", "these strings are almos equal", "not the same at all", None, None,
                      "", "a", "smithe", "unicode", "a\U0001F600c", "MARHTA", "DUANE", "DICKSONX", "cba", "y"]})
    floats = pd.DataFrame({"float_col_l": [1.0, 100.0, 100.0, -100.0, None, 0.0, 0.0, 5.0],
                           "float_col_r": [1.0, 99.9, 90.1, -85.1, -85.1, 0.0, 1.0, -5.0]})
    to_table(con, strs, "str_comp")
    to_table(con, floats, "float_comp")
    out = {"str_comp": frame_json(strs), "float_comp": frame_json(floats), "cases": []}
    str_cases = [
        ("strict_equality_2", sql_gen_case_smnt_strict_equality_2("str_col", "str_col")),
        ("levenshtein_3", sql_gen_case_stmt_levenshtein_3("str_col", "str_col")),
        ("levenshtein_4", sql_gen_case_stmt_levenshtein_4("str_col", "str_col")),
        ("jaro_2", sql_gen_gammas_case_stmt_jaro_2("str_col", "str_col")),
        ("jaro_3", sql_gen_gammas_case_stmt_jaro_3("str_col", "str_col")),
        ("jaro_4_t3_0.001", sql_gen_gammas_case_stmt_jaro_4("str_col", "str_col", threshold3=0.001)),
        ("jaro_4", sql_gen_gammas_case_stmt_jaro_4("str_col", "str_col")),
        ("literal_hi", "case  when str_col_l = str_col_r then 2 when str_col_l = 'hi' then 1 else 0 end as gamma_str_col"),
    ]
    float_cases = [
        ("numeric_2", sql_gen_case_stmt_numeric_2("float_col", "float_col")),
        ("numeric_abs_3", sql_gen_case_stmt_numeric_abs_3("float_col", "float_col", abs_amount=1)),
        ("numeric_abs_4", sql_gen_case_stmt_numeric_abs_4("float_col", "float_col", abs_amount_low=1, abs_amount_high=10)),
        ("numeric_perc_3_0.01", sql_gen_case_stmt_numeric_perc_3("float_col", "float_col", per_diff=0.01)),
        ("numeric_perc_3_0.2", sql_gen_case_stmt_numeric_perc_3("float_col", "float_col", per_diff=0.20)),
        ("numeric_perc_4", sql_gen_case_stmt_numeric_perc_4("float_col", "float_col", per_diff_low=0.01, per_diff_high=0.1)),
    ]
    for name, sql in str_cases:
        lv = [r[0] for r in con.execute(f"select {sql} from str_comp").fetchall()]
        out["cases"].append({"name": name, "table": "str_comp", "case_expression": sql, "levels": lv})
    for name, sql in float_cases:
        lv = [r[0] for r in con.execute(f"select {sql} from float_comp").fetchall()]
        out["cases"].append({"name": name, "table": "float_comp", "case_expression": sql, "levels": lv})
    names = pd.DataFrame([  # reference tests/test_spark.py:388-406
        ("smith", "john", "david", "smith", "john", "david"),
        ("smith", "john", "david", "smithe", "john", "david"),
        ("smith", "john", "david", "john", "smith", "david"),
        ("smith", "john", "david", "john", "david", "smithe"),
        ("linacre", "john", "david", "linaker", "john", "david"),
        ("smith", "john", "david", "john", "david", "smarty"),
        ("smith", "john", None, "jones", "smith", None),
    ], columns=["surname_l", "forename1_l", "forename2_l", "surname_r", "forename1_r", "forename2_r"])
    to_table(con, names, "df_names")
    sql = sql_gen_gammas_name_inversion_4("surname", ["forename1", "forename2"], "surname")
    lv = [r[0] for r in con.execute(f"select {sql} from df_names").fetchall()]
    out["names"] = frame_json(names)
    out["cases"].append({"name": "name_inversion_4", "table": "df_names", "case_expression": sql, "levels": lv})
    return out


def string_values():
    pairs = [("smith", "smithe"), ("linacre", "linaker"), ("these strings are almost equal", "not the same at all"),
             ("", ""), ("", "a"), ("a", ""), ("a", "a"), ("ab", "ba"), ("MARTHA", "MARHTA"), ("DWAYNE", "DUANE"),
             ("DIXON", "DICKSONX"), ("JELLYFISH", "SMELLYFISH"), ("crate", "trace"), ("abcdefghij", "abcdefghij"),
             ("Ünïcødé", "Unicode"), ("a\U0001F600b", "a\U0001F600c"), ("\U0001F600", "\U0001F601"),
             ("ß", "ss"), ("aaaa", "aaab"), ("abcabcabc", "cbacbacba"), ("x" * 70, "x" * 69 + "y"),
             ("the quick brown fox jumps over the lazy dog and keeps running far away", "the quick brown fox"),
             ("1234", "smith"), ("john", "1234")]
    rng = np.random.Generator(np.random.PCG64(11))
    alpha = list("abcde") + ["é", "\U0001D400"]
    for _ in range(300):
        a = "".join(rng.choice(alpha, size=int(rng.integers(0, 14))))
        b = "".join(rng.choice(alpha, size=int(rng.integers(0, 14))))
        pairs.append((a, b))
    return {"pairs": [[a, b] for a, b in pairs],
            "jw": [py_jaro_winkler(a, b) for a, b in pairs],
            "lev": [py_levenshtein(a, b) for a, b in pairs]}


def custom_settings():
    return {
        "link_type": "dedupe_only", "proportion_of_matches": 0.2, "max_iterations": 4,
        "blocking_rules": ["l.city = r.city", "l.surname = r.surname AND l.first_name = r.first_name"],
        "additional_columns_to_retain": ["cluster"],
        "comparison_columns": [
            {"custom_name": "name_inversion", "custom_columns_used": ["surname", "first_name"], "num_levels": 4,
             "case_expression": sql_gen_gammas_name_inversion_4("surname", ["first_name"], "name_inversion")},
            {"col_name": "first_name", "num_levels": 4},
            {"col_name": "age", "data_type": "numeric", "num_levels": 3},
            {"col_name": "email", "num_levels": 4, "case_expression": sql_gen_case_stmt_levenshtein_4("email", "email")},
            {"col_name": "dob", "num_levels": 3, "case_expression":
                "CASE WHEN dob_l IS NULL OR dob_r IS NULL THEN -1 WHEN dob_l = dob_r THEN 2 "
                "WHEN substr(dob_l, 1, 7) = substr(dob_r, 1, 7) OR jaro_winkler_sim(dob_l, dob_r) >= 0.9 THEN 1 "
                "ELSE 0 END"},
        ],
    }


def tiny_numbers_settings(max_iterations):  # reference tests/test_spark.py:137-150
    return {
        "link_type": "dedupe_only", "proportion_of_matches": 0.4,
        "comparison_columns": [
            {"col_name": "mob", "num_levels": 2,
             "m_probabilities": [5.9380419956766985e-25, 1 - 5.9380419956766985e-25], "u_probabilities": [0.8, 0.2]},
            {"col_name": "surname", "num_levels": 2}],
        "blocking_rules": ["l.mob = r.mob", "l.surname = r.surname"],
        "max_iterations": max_iterations,
    }


def edge_cases():
    """Reference edge cases replayed as fixtures (VERDICT r1 'missing' 5)."""
    out = {}
    # first E-step with the settings' m / u (max_iterations = 0): the literal lists of
    # tests/test_expectation.py:57-66 and tests/test_nulls.py:11
    st = gamma_settings_1()
    st["max_iterations"] = 0
    g = reference_pipeline(st, False, df=test1_records(), ll=True)
    want = [0.893617021, 0.705882353, 0.705882353, 0.189189189, 0.189189189, 0.893617021, 0.375, 0.375]
    assert all(abs(a - b) < 1e-8 for a, b in zip(g["df_e"]["match_probability"], want)), g["df_e"]["match_probability"]
    g["reference_literal_mp"] = want
    out["first_estep_test1"] = g
    st = gamma_settings_2()
    st["max_iterations"] = 0
    g = reference_pipeline(st, False, df=test2_records(), ll=True)
    want = [0.322580645, 0.16, 0.1, 0.16, 0.1, 0.1]
    assert all(abs(a - b) < 1e-8 for a, b in zip(g["df_e"]["match_probability"], want)), g["df_e"]["match_probability"]
    g["reference_literal_mp"] = want
    out["first_estep_nulls"] = g
    # tests/test_spark.py:130-160 (m = 5.9e-25 through the 35-digit literal), the first E-step and 3 iterations
    out["tiny_numbers_estep"] = reference_pipeline(tiny_numbers_settings(0), False, df=test1_records(), ll=True)
    out["tiny_numbers_em"] = reference_pipeline(tiny_numbers_settings(3), False, df=test1_records(), ll=True)
    # compute_ll through every iteration (expectation_step.py:52-57, 224-272)
    out["ll_test1"] = reference_pipeline(gamma_settings_1(), False, df=test1_records(), ll=True)
    out["ll_nulls"] = reference_pipeline(gamma_settings_2(), False, df=test2_records(), ll=True)
    df1 = make_records(**CONFIGS[1])
    out["ll_cfg1"] = reference_pipeline(cfg_settings(1, max_iterations=4), True,
                                        df=df1[["unique_id", "first_name", "surname", "dob", "city", "email"]], ll=True)
    # NULL unique ids: `l.uid < r.uid` is NULL, so same-source pairs with a NULL id are dropped
    # (blocking.py:136, :139); link_and_dedupe keeps cross-source pairs through `l.src < r.src`
    recs = pd.DataFrame({"unique_id": [1.0, None, 3.0, None, 5.0, 2.0],
                         "surname": ["a", "a", "a", "b", "b", "a"], "first_name": ["x", "y", "x", "y", "x", "y"]})
    st = {"link_type": "dedupe_only", "comparison_columns": [{"col_name": "first_name"}],
          "blocking_rules": ["l.surname = r.surname"], "max_iterations": 1}
    out["null_uid_dedupe"] = reference_pipeline(st, False, df=recs)
    st = {"link_type": "link_and_dedupe", "comparison_columns": [{"col_name": "first_name"}, {"col_name": "surname"}],
          "blocking_rules": ["l.surname = r.surname"], "max_iterations": 1}
    out["null_uid_link_and_dedupe"] = reference_pipeline(st, False, df_l=recs.iloc[:3].reset_index(drop=True),
                                                         df_r=recs.iloc[3:].reset_index(drop=True))
    return out


def main():
    # 1. conftest test1 (two EM iterations, substr custom expression), jaro off (spark="supress_warnings")
    dump("test1", reference_pipeline(gamma_settings_1(), False, df=test1_records()))
    # 2. test_main_api settings with and without the jar's JW
    s = {"link_type": "dedupe_only", "comparison_columns": [{"col_name": "surname"}, {"col_name": "mob"}],
         "blocking_rules": ["l.mob = r.mob", "l.surname = r.surname"], "max_iterations": 2}
    dump("main_api_nojaro", reference_pipeline(s, False, df=test1_records()))
    s = {"link_type": "dedupe_only", "blocking_rules": ["l.mob = r.mob", "l.surname = r.surname"],
         "comparison_columns": [{"col_name": "surname", "num_levels": 3},
                                {"col_name": "mob", "case_expression": sql_gen_case_smnt_strict_equality_2("mob")}],
         "max_iterations": 3}
    dump("main_api_jaro", reference_pipeline(s, True, df=test1_records()))
    # 3. nulls, cartesian
    dump("test2_nulls", reference_pipeline(gamma_settings_2(), False, df=test2_records()))
    # 4. known data-generating process, EM only from a gamma table
    dump("dgp", reference_pipeline(gamma_settings_4(), False, df_gammas=dgp_gammas()))
    # 5. blocking / link options
    cases = {}
    base_cols = [{"col_name": "first_name"}, {"col_name": "surname"}]
    rules2 = ["l.first_name = r.first_name", "l.surname = r.surname"]
    for repeat in (False, True):
        l, r = link_data(repeat)
        for lt in ("link_only", "link_and_dedupe"):
            for rules in (rules2, []):
                st = {"link_type": lt, "comparison_columns": copy.deepcopy(base_cols), "blocking_rules": rules,
                      "max_iterations": 2}
                cases[f"{lt}_{'repeat' if repeat else 'plain'}_{'rules' if rules else 'cartesian'}"] = \
                    reference_pipeline(st, False, df_l=l, df_r=r)
        st = {"link_type": "dedupe_only", "comparison_columns": copy.deepcopy(base_cols), "blocking_rules": rules2,
              "max_iterations": 2}
        cases[f"dedupe_only_{'repeat' if repeat else 'plain'}_rules"] = reference_pipeline(st, False, df=l)
    st = {"link_type": "dedupe_only", "comparison_columns": copy.deepcopy(base_cols),
          "blocking_rules": ["l.surname = r.surname", "l.first_name = r.first_name"], "max_iterations": 1}
    cases["blocks_dedupe"] = reference_pipeline(st, True, df=blocks_records())
    dump("link_options", cases)
    # 6. comparison templates, level tables and raw JW / Levenshtein values
    dump("case_levels", case_level_tables())
    dump("string_values", string_values())
    # 7. synthetic config-1 look-alike (1k records, 10 EM iterations)
    df1 = make_records(**CONFIGS[1])
    dump("synthetic_cfg1", reference_pipeline(cfg_settings(1), True, df=df1[["unique_id", "first_name", "surname",
                                                                              "dob", "city", "email"]]))
    # 8. custom expressions / numeric / additional columns on synthetic data
    df2 = make_records(400, seed=5, surname_vocab=40, first_vocab=60, city_vocab=150)
    df2["age"] = (df2["cluster"] % 60 + 18).astype(float)
    df2.loc[df2.index % 13 == 0, "age"] = np.nan
    dump("custom_exprs", reference_pipeline(custom_settings(), True, df=df2))
    # 9. link_only with term-frequency adjustment on surname (config-3 look-alike, small)
    df3 = make_records(500, seed=9, surname_vocab=60, first_vocab=80, city_vocab=20)
    left = df3[df3.index % 2 == 0].reset_index(drop=True)
    right = df3[df3.index % 2 == 1].reset_index(drop=True)
    left["unique_id"] = np.arange(len(left))
    right["unique_id"] = np.arange(len(right))
    st = cfg_settings(1, max_iterations=5)
    st["link_type"] = "link_only"
    st["retain_matching_columns"] = True
    st["retain_intermediate_calculation_columns"] = True
    st["blocking_rules"] = ["l.surname = r.surname", "l.dob = r.dob", "l.email = r.email"]
    st["comparison_columns"][1]["term_frequency_adjustments"] = True
    st["em_convergence"] = 1e-4
    dump("link_tf", reference_pipeline(st, True, df_l=left, df_r=right, tf=True))
    # 10. edge cases, log-likelihood, NULL unique ids
    dump("edge_cases", edge_cases())


def main_edge_only():
    dump("edge_cases", edge_cases())


if __name__ == "__main__":
    if "--edge-only" in sys.argv:
        main_edge_only()
    else:
        main()
