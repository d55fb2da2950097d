"""Host-side logic that needs no GPU: settings completion, the SQL compiler, Params, M-step algebra."""
import copy
import json
import math
import os
import warnings

import numpy as np
import pytest

import oracle as orc
from conftest import load_golden

from splink_amd import case_statements as cs
from splink_amd.compiler import Schema, compile_comparisons, compile_rule
from splink_amd.engine import N_HEAD, m_step_rows
from splink_amd.params import Params, load_params_from_json
from splink_amd.session import AmdSession
from splink_amd.settings import complete_settings_dict
from splink_amd.sqlexpr import Bin, Case, Col, Func, Lit, parse
from splink_amd.validate import ValidationError, validate_settings

warnings.filterwarnings("ignore")
GOLDENS = ["test1", "main_api_nojaro", "main_api_jaro", "test2_nulls", "synthetic_cfg1", "custom_exprs", "link_tf"]


def spark_for(jaro):
    return AmdSession(0) if jaro else "supress_warnings"


@pytest.mark.parametrize("name", GOLDENS)
def test_settings_completion_matches_reference(name):
    g = load_golden(name)
    ours = complete_settings_dict(copy.deepcopy(g["settings_in"]), spark_for(g["jaro"]))
    ref = g["settings_completed"]
    for k in ("em_convergence", "unique_id_column_name", "additional_columns_to_retain", "retain_matching_columns",
              "retain_intermediate_calculation_columns", "max_iterations", "proportion_of_matches", "link_type"):
        assert ours[k] == ref[k], k
    forms = {}
    for key in ("df", "df_l"):
        if key in g:
            for c, vals in g[key].items():
                forms[c] = "num" if all(v is None or isinstance(v, (int, float)) for v in vals) else "str"
    schema = Schema(forms)
    for a, b in zip(ours["comparison_columns"], ref["comparison_columns"]):
        for k in ("gamma_index", "num_levels", "data_type", "term_frequency_adjustments"):
            assert a[k] == b[k]
        assert a["m_probabilities"] == pytest.approx(b["m_probabilities"], rel=1e-15)
        assert a["u_probabilities"] == pytest.approx(b["u_probabilities"], rel=1e-15)
    # our template text and the reference's compile to the same device program
    pa = compile_comparisons(ours, schema)
    pb = compile_comparisons(ref, schema)
    assert (pa.programs == pb.programs).all()
    assert (pa.instrs == pb.instrs).all()
    assert pa.operands == pb.operands and pa.literals == pb.literals


def test_params_layout_and_json_roundtrip(tmp_path):
    g = load_golden("test1")
    p = Params(copy.deepcopy(g["settings_in"]), "supress_warnings")
    assert list(p.params["π"]["gamma_mob"].keys()) == ["gamma_index", "desc", "column_name", "custom_comparison",
                                                        "num_levels", "prob_dist_match", "prob_dist_non_match"]
    rows = g["iterations"][0]["pi_rows"]
    p._update_params(g["iterations"][0]["lambda"], rows)
    assert p.params["π"]["gamma_mob"]["prob_dist_match"]["level_0"]["probability"] == \
        g["iterations"][0]["pi"]["gamma_mob"]["m"][0]
    assert len(p.param_history) == 1 and p.iteration == 2
    path = tmp_path / "m.json"
    p.save_params_to_json_file(str(path))
    with pytest.raises(ValueError):
        p.save_params_to_json_file(str(path))
    q = load_params_from_json(str(path))
    assert q.params == json.loads(json.dumps(p.params))
    assert q.iteration == 1  # the reference does not restore the iteration counter (params.py:569-573)
    d = json.load(open(path))
    assert set(d) == {"current_params", "historical_params", "settings"}


def _stats_from_histogram(gam, nlev, lam, m, u):
    """Product statistics layout from the oracle's per-pair statistics (test helper)."""
    s = orc.em_stats(gam, nlev, lam, m, u)
    out = [s[0], s[1], s[2], 0.0, 0.0]
    return np.array(out + list(s[3:]))


@pytest.mark.parametrize("name", ["test1", "test2_nulls", "synthetic_cfg1"])
def test_m_step_rows_match_reference_rows(name):
    g = load_golden(name)
    st = g["settings_completed"]
    names = [f"gamma_{c.get('custom_name', c.get('col_name'))}" for c in st["comparison_columns"]]
    nlev = [c["num_levels"] for c in st["comparison_columns"]]
    gam = np.array([g["gammas"][n] for n in names], dtype=np.int8).T
    m = [g["initial"]["pi"][n]["m"] for n in names]
    u = [g["initial"]["pi"][n]["u"] for n in names]
    stats = _stats_from_histogram(gam, nlev, g["initial"]["lambda"], m, u)
    lam, rows = m_step_rows(stats, names, nlev)
    it = g["iterations"][0]
    assert lam == pytest.approx(it["lambda"], rel=1e-9)
    key = lambda r: (r["gamma_col"], r["gamma_value"])
    exp = sorted(it["pi_rows"], key=key)
    got = sorted(rows, key=key)
    assert [key(r) for r in got] == [key(r) for r in exp]
    for a, b in zip(got, exp):
        for k in ("new_probability_match", "new_probability_non_match"):
            assert (a[k] is None) == (b[k] is None)
            if a[k] is not None:
                assert a[k] == pytest.approx(b[k], rel=1e-9)


def test_parser_basics():
    e = parse("case when a_l is null or a_r is null then -1 when a_l = a_r then 1 else 0 end as gamma_a")
    assert isinstance(e, Case) and len(e.whens) == 2 and e.else_ == Lit(0)
    assert parse("substr(x_l, 1, 3)") == Func("substr", (Col("x_l"), Lit(1), Lit(3)))
    assert parse("l.first_name = r.first_name") == Bin("=", Col("first_name", "l"), Col("first_name", "r"))
    assert parse("'it''s'") == Lit("it's")
    with pytest.raises(ValueError):
        parse("case when a = then 1 end")


def test_compiler_rejects_unsupported_sql():
    schema = Schema({"a": "str", "b": "num"})
    bad = [
        "case when a_l is null then -1 when initcap(a_l) = initcap(a_r) then 1 else 0 end",
        "case when a_l = a_r then 1 end",  # no ELSE
        "case when a_l = a_r then 5 else 0 end",  # level out of range for 2 levels
        "case when a_l like 'x%' then 1 else 0 end",
    ]
    for expr in bad:
        st = {"comparison_columns": [{"col_name": "a", "num_levels": 2, "case_expression": expr}]}
        with pytest.raises(ValueError):
            compile_comparisons(st, schema)
    with pytest.raises(ValueError):
        compile_rule("l.a < r.a", schema)
    with pytest.raises(ValueError):
        compile_rule("l.a = l.a", schema)


def test_blocking_rule_compile():
    schema = Schema({"surname": "str", "dob": "str", "first_name": "str"})
    r = compile_rule("l.surname = r.surname AND substr(l.dob,1,4) = substr(r.dob,1,4)", schema)
    assert r.symmetric and len(r.terms) == 2
    r = compile_rule("l.first_name = r.surname", schema)
    assert not r.symmetric


def test_validation_errors():
    with pytest.raises(ValidationError):
        validate_settings({"link_type": "dedupe", "comparison_columns": [{"col_name": "a"}]})
    with pytest.raises(ValidationError):
        validate_settings({"link_type": "dedupe_only", "comparison_columns": []})
    with pytest.raises(ValidationError):
        validate_settings({"link_type": "dedupe_only", "comparison_columns": [{"col_name": "a", "bogus": 1}]})
    validate_settings({"link_type": "dedupe_only", "comparison_columns": [{"col_name": "a"}]})


def test_jaro_detection():
    assert cs._check_jaro_registered(None) is False
    assert cs._check_jaro_registered("supress_warnings") is False
    assert cs._check_jaro_registered(AmdSession(0)) is True


def test_derived_column_programs():
    """Spark built-ins over one record (lower / upper / trim / concat / cast) compile to derived columns
    (splink_amd/derived.py): lower(a_l) and lower(a_r) name one column; a null guard on the input column is
    moved onto the derived one when every test reads a through the same lower / upper / trim chain."""
    from splink_amd.compiler import _guard_on_derived
    schema = Schema({"a": "str", "b": "str", "n": "num"})
    expr = ("case when a_l is null or a_r is null then -1 "
            "when jaro_winkler_sim(lower(a_l), lower(a_r)) > 0.9 then 1 else 0 end")
    p = compile_comparisons({"comparison_columns": [{"col_name": "a", "num_levels": 2, "case_expression": expr}]},
                            schema)
    assert list(p.derived) == ["lower(a)"] and p.columns == [("lower(a)", "str")]
    t = _guard_on_derived(parse(expr))
    assert t.whens[0][0] == Bin("or", parse("lower(a_l) is null"), parse("lower(a_r) is null"))
    # two different chains, or a bare reference: the guard stays
    for e in ["case when a_l is null or a_r is null then -1 when lower(a_l) = upper(a_r) then 1 else 0 end",
              "case when a_l is null or a_r is null then -1 when lower(a_l) = a_r then 1 else 0 end"]:
        assert _guard_on_derived(parse(e)) == parse(e)
    # cast / concat / implicit casts folded into the derived expression
    e2 = ("case when cast(n_l as string) = concat(b_r, 'x') then 1 "
          "when jaro_winkler_sim(cast(a_l as int), cast(a_r as int)) > 0.5 then 1 else 0 end")
    p = compile_comparisons({"comparison_columns": [{"col_name": "a", "num_levels": 2, "case_expression": e2}]},
                            schema)
    assert set(p.derived) == {"cast(n as string)", "concat(b, 'x')", "cast(cast(a as int) as string)"}
    for bad in ["case when lower(a_l) = lower(a_l || a_r) then 1 else 0 end",
                "case when concat(a_l, b_r) = 'x' then 1 else 0 end",  # mixes the two records
                "case when cast(a_l as date) = cast(a_r as date) then 1 else 0 end",
                "case when lower('x') = a_l then 1 else 0 end"]:  # no column
        with pytest.raises(ValueError):
            compile_comparisons({"comparison_columns": [{"col_name": "a", "num_levels": 2, "case_expression": bad}]},
                                schema)


def test_derived_values_match_oracle_functions():
    """Each derived expression evaluated on the host (product, once per row) equals the oracle's sqlite
    evaluation with its Spark-semantic functions; string-only expressions go through pyarrow kernels on
    ASCII columns and the per-row path otherwise."""
    import pandas as pd
    from splink_amd import derived as D
    rng = np.random.Generator(np.random.PCG64(9))
    words = np.array(["Anna", " anna ", "ANNA", "", "  ", "O'Neil", "Straße", "İlker", "Zoë", "x y"], dtype=object)
    nums = np.array(["12", " 12", "12.9", "-0", "+13", "1e1", "abc", "", "99999999999", "7.", ".5", "-12.5",
                     "1.8d", " 1.8 ", "Infinity", "-Infinity", "0x1p3", "0X1.Cp0", "+.5", "-", ".",
                     # double -> smallint / tinyint saturates at the int range, then wraps (Cast.castToShort);
                     # a suffix after Infinity / NaN does not parse (NULL)
                     "40000.5", "-40000", "1e10", "300.7", "-1e300", "Infinityd", "NaNf"], dtype=object)
    n = 400
    df = pd.DataFrame({"a": rng.choice(words, n), "b": rng.choice(words[:6], n), "n": rng.choice(nums, n)})
    for c in df.columns:
        df.loc[rng.random(n) < 0.1, c] = None
    df_arrow = df.astype({"b": pd.ArrowDtype(__import__("pyarrow").large_string())})
    exprs = ["lower(a)", "upper(trim(a))", "ltrim(a)", "rtrim(b)", "concat(a, ' ', b)", "concat_ws('|', a, b, n)",
             "cast(n as int)", "cast(n as bigint)", "cast(n as smallint)", "cast(n as double)",
             "cast(cast(n as double) as int)", "cast(cast(n as double) as smallint)",
             "cast(cast(n as double) as tinyint)", "cast(cast(n as double) as bigint)", "substr(lower(a), 2, 3)", "lower(ifnull(a, b))", "upper(b)",
             "concat(b, '-', b)", "trim(b)"]
    con = orc.connect()
    df.to_sql("t", con, index=False)
    schema = Schema({"a": "str", "b": "str", "n": "str"})
    for e in exprs:
        node, _ = D.neutralise(parse(e), lambda c: (c.name, 0))
        form = D.form_of(node, schema.form)
        want = [r[0] for r in con.execute(f"select {orc.rewrite_casts(e)} from t").fetchall()]
        for frame in (df, df_arrow):
            got = D.evaluate(node, frame, form)
            got = [None if (x is None or x is pd.NA or (isinstance(x, float) and math.isnan(x))) else x
                   for x in got.tolist()]
            if form == "num":
                want_n = [None if w is None else float(w) for w in want]
                assert got == want_n, (e, [(g, w) for g, w in zip(got, want_n) if g != w][:5])
            else:
                assert got == want, (e, [(g, w) for g, w in zip(got, want) if g != w][:5])


def test_float64_encoding_keeps_infinities():
    """Numeric columns go to the device as fp64 + validity: NaN / None are NULL, +-Infinity stay infinite
    (Spark doubles; abs(Infinity - Infinity) is NaN, so `< t` is false, not true as for clamped values)."""
    import pandas as pd
    from splink_amd.table import encode_float64
    vals, valid = encode_float64(pd.Series([1.5, float("inf"), -float("inf"), float("nan"), None]))
    assert valid.tolist() == [1, 1, 1, 0, 0]
    assert vals[1] == float("inf") and vals[2] == -float("inf") and vals[3] == 0.0


def test_spark_builtins_match_oracle_functions():
    """soundex / regexp_replace / regexp_extract / to_date / date_add / date_sub / datediff as derived columns
    (derived.py, evaluated per row at ingest) equal the oracle's independent restatements in sqlite, on names,
    punctuation, non-ASCII text and date strings in every shape stringToDate accepts or rejects (dates from 1583
    on: before that the reference's hybrid calendar is Julian, parity unpinned)."""
    import pandas as pd
    from splink_amd import derived as D
    words = ["Robert", "Rupert", "Rubin", "Ashcraft", "Tymczak", "Pfister", "Honeyman", "", "  x", "élan", "O'Hara",
             "1abc", "Lee", "Gutierrez", "a-b-c", "Wh", None]
    dates = ["2020-01-15", "2020-1-5", "2020", "2020-02-30", "1999-12-31 10:00", "2000-02-29T01:02", "20200101",
             " 2021-03-04 ", "x", "", "1600-03-01", "2020-13-01", "2020-", "2020-05", "1970-01-01", None, "2021-02-29"]
    df = pd.DataFrame({"a": words, "d": dates})
    con = orc.connect()
    df.to_sql("t", con, index=False)
    exprs = ["soundex(a)", "soundex(lower(a))", "regexp_replace(a, '[aeiou]', '')", "regexp_replace(a, '(r)(u)', '$2$1')",
             "regexp_extract(a, '([A-Z])([a-z]+)', 2)", "regexp_extract(a, 'x(y)?', 1)", "regexp_extract(a, '([a-z]+)')",
             "regexp_replace(a, '\\\\d', '#')", "regexp_replace(a, 'a*', '-')", "regexp_replace(a, '(.)', '\\\\$$1')",
             "cast(to_date(d) as string)", "datediff(d, '2020-01-01')", "cast(date_add(d, 40) as string)",
             "datediff(date_sub(d, 3), '1970-01-01')", "datediff(to_date(d), to_date(d))"]
    schema = Schema({"a": "str", "d": "str"})
    for e in exprs:
        node, _ = D.neutralise(parse(e), lambda c: (c.name, 0))
        form = D.form_of(node, schema.form)
        want = [r[0] for r in con.execute(f"select {orc.rewrite_casts(orc.spark_literals(e))} from t").fetchall()]
        got = D.evaluate(node, df, form)
        got = [None if (x is None or x is pd.NA or (isinstance(x, float) and math.isnan(x))) else x for x in got.tolist()]
        if form == "num":
            want = [None if w is None else float(w) for w in want]
        assert got == want, (e, [(r, g, w) for r, g, w in zip(df.to_dict("records"), got, want) if g != w][:4])
    # American Soundex reference values (H / W do not separate equal codes, vowels do)
    assert [D.spark_soundex(x) for x in ["Robert", "Rupert", "Rubin", "Ashcraft", "Tymczak", "Pfister", "Honeyman"]] == \
        ["R163", "R163", "R150", "A261", "T522", "P236", "H555"]
    assert D.spark_string_to_date("1970-01-01") == 0 and D.day_to_string(D.epoch_day(1582, 10, 15) - 1) == "1582-10-04"


def test_datediff_compiles_to_day_columns():
    """abs(datediff(a_l, a_r)) <= t is ABSDIFF over the derived day-number column datediff(a, '1970-01-01'); a
    signed datediff(a_l, a_r) cmp t is NUM_CMP against b's column shifted by t days (date_add), a non-integral t
    first rounded to the integral threshold with the same truth value."""
    from splink_amd import _native as N
    schema = Schema({"a": "str", "b": "str"})
    case = ("case when a_l is null or a_r is null then -1 when abs(datediff(a_l, a_r)) <= 30 then 3 "
            "when datediff(a_l, b_r) > 365 then 2 when 10.5 >= datediff(b_l, a_r) then 1 else 0 end")
    prog = compile_comparisons({"comparison_columns": [{"col_name": "a", "num_levels": 4, "case_expression": case}]},
                               schema)
    assert set(prog.derived) == {"datediff(a, '1970-01-01')", "datediff(date_add(b, 365), '1970-01-01')",
                                 "datediff(b, '1970-01-01')", "datediff(date_add(a, 10), '1970-01-01')"}
    ops = [i[0] for i in prog.instrs]
    assert N.OP["ABSDIFF"] in ops and ops.count(N.OP["NUM_CMP"]) == 2
    for bad in ["case when datediff(a_l, a_r) = 1.5 then 1 else 0 end",
                "case when regexp_replace(a_l, b_l, '') = a_r then 1 else 0 end",
                "case when regexp_replace(a_l, '(x', '') = a_r then 1 else 0 end",
                "case when regexp_replace(a_l, 'x++', '') = a_r then 1 else 0 end",
                "case when regexp_extract(a_l, '(x)', 2) = a_r then 1 else 0 end",
                "case when regexp_extract(a_l, 'x') = a_r then 1 else 0 end",
                "case when regexp_replace(a_l, '(x)', '$2') = a_r then 1 else 0 end",
                "case when date_add(a_l, b_l) = a_r then 1 else 0 end",
                "case when to_date(a_l, 'yyyy') = a_r then 1 else 0 end"]:
        with pytest.raises(ValueError):
            compile_comparisons({"comparison_columns": [{"col_name": "a", "num_levels": 2, "case_expression": bad}]},
                                schema)


def test_string_literals_unescape_as_spark():
    """Backslash escapes in string literals as Spark's parser reads them (ParserUtils.unescapeSQLString); a doubled
    quote is one quote."""
    from splink_amd.sqlexpr import unescape_literal
    cases = {"'abc'": "abc", "'it''s'": "it's", "'\\d+'": "d+", "'\\\\d+'": "\\d+", "'a\\nb'": "a\nb",
             "'\\u0041x'": "Ax", "'\\101'": "A", "'\\%'": "\\%", "'\\''": "'", "'\\q'": "q", "'\\Z'": "\x1a"}
    for q, want in cases.items():
        assert unescape_literal(q) == want, q
        assert parse(f"a_l = {q}").b.value == want
    for q in cases:
        sql = orc.spark_literals(f"select {q}")
        assert orc.connect().execute(sql).fetchone()[0] == cases[q], q
