"""Spark built-ins over one record inside case_expressions, on the HIP path, against the sqlite oracle.

The reference splices each completed case_expression verbatim into Spark SQL (gammas.py:47, :53;
case_statements.py:24-43 lower-cases it first), so `lower` / `upper` / `trim` / `ltrim` / `rtrim` /
`concat` / `concat_ws` / `cast` work around the `_l` / `_r` operands, also under `jaro_winkler_sim` and
`levenshtein`.  The device evaluates each such sub-expression once per row (splink_amd/derived.py) and
compares the derived columns like input columns; the oracle evaluates the whole CASE per pair in sqlite
with Spark-semantic functions (oracle.connect / rewrite_casts).  ASCII rows are pinned by that restatement
of Spark; the non-ASCII rows (É, ß, İ) follow Python's Unicode case mapping on both sides -- "parity
unpinned" against Java's toLowerCase / toUpperCase, kept to exercise the UTF-16 path of derived columns.
"""
import copy

import numpy as np
import pandas as pd
import pytest

import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd():
    from splink_amd import AmdSession, _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    return AmdSession(0)


def _frame(n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    first = np.array(["Anna", "anna", " Anna ", "ANNA", "Ann", "Jon", "john", "JOHN ", "Éloïse", "éloïse", "Straße",
                      "STRASSE", "İlker", "ilker", "Zoë", "", "  "], dtype=object)
    last = np.array(["Smith", "smith", "SMITHE", "Smyth", " Jones", "jones", "O'Neil", "o'neil", "Müller",
                     "MÜLLER", "Brown", "brown "], dtype=object)
    ages = np.array(["12", " 12", "12.9", "-0", "13", "+13", "1e1", "abc", "", "99999999999", "7.", ".5", "-12.5"],
                    dtype=object)
    heights = np.array(["1.80", " 1.8 ", "1.8d", "180e-2", "Infinity", "-Infinity", "x", "2", "1.75", "0x1p0",
                        "0X1.Cp0", "0x1p3f", ".5e1"], dtype=object)
    df = pd.DataFrame({
        "unique_id": np.arange(n, dtype=np.int64),
        "first_name": rng.choice(first, n),
        "surname": rng.choice(last, n),
        "age": rng.choice(ages, n),
        "height": rng.choice(heights, n),
        "city": rng.choice(np.array(["a", "b", "c", "d", "e"], dtype=object), n),
        "visit": _visits(rng, n),
    })
    for c in ["first_name", "surname", "age", "height", "visit"]:
        df.loc[rng.random(n) < 0.07, c] = None
    return df


def _visits(rng, n):
    """Date strings as a source hands them over: ISO dates, unpadded months / days, a year alone, times after
    the date, surrounding spaces, and strings that are not dates (NULL for to_date / datediff)."""
    base = np.datetime64("2019-06-01") + rng.integers(0, 900, n).astype("timedelta64[D]")
    out = np.array([str(d) for d in base], dtype=object)
    odd = rng.random(n)
    for i in np.nonzero(odd < 0.25)[0]:
        y, m, d = str(base[i]).split("-")
        out[i] = rng.choice([f"{y}-{int(m)}-{int(d)}", f"{y}-{m}-{d} 10:30:00", f"{y}-{m}-{d}T08:00", f" {y}-{m}-{d} ",
                             f"{y}-{m}", y, "2020-02-30", "20200101", "soon", ""])
    return out


EXPRS = [
    # a template-shaped JW column over a derived column (the filter path)
    ("fn_jw", ["first_name"], 3,
     "case when first_name_l is null or first_name_r is null then -1 "
     "when jaro_winkler_sim(lower(first_name_l), lower(first_name_r)) > 0.94 then 2 "
     "when jaro_winkler_sim(lower(first_name_l), lower(first_name_r)) > 0.88 then 1 else 0 end"),
    ("fn_trim", ["first_name"], 3,
     "case when lower(trim(first_name_l)) is null or lower(trim(first_name_r)) is null then -1 "
     "when lower(trim(first_name_l)) = lower(trim(first_name_r)) then 2 "
     "when ltrim(first_name_l) = ltrim(first_name_r) or rtrim(first_name_l) = rtrim(first_name_r) then 1 "
     "else 0 end"),
    ("sn_lev", ["surname"], 4,
     "case when surname_l is null or surname_r is null then -1 "
     "when upper(surname_l) = upper(surname_r) then 3 "
     "when levenshtein(upper(trim(surname_l)), upper(trim(surname_r))) <= 1 then 2 "
     "when levenshtein(lower(surname_l), lower(surname_r))/((length(lower(surname_l)) + "
     "length(lower(surname_r)))/2) <= 0.4 then 1 else 0 end"),
    ("full", ["first_name", "surname"], 3,
     "case when concat(first_name_l, ' ', surname_l) is null or concat(first_name_r, ' ', surname_r) is null "
     "then -1 when concat_ws('|', lower(first_name_l), lower(surname_l)) = "
     "concat_ws('|', lower(first_name_r), lower(surname_r)) then 2 "
     "when jaro_winkler_sim(concat(first_name_l, ' ', surname_l), concat(first_name_r, ' ', surname_r)) > 0.8 "
     "then 1 else 0 end"),
    ("age", ["age"], 3,
     "case when cast(age_l as int) is null or cast(age_r as int) is null then -1 "
     "when cast(age_l as int) = cast(age_r as int) then 2 "
     "when abs(cast(age_l as bigint) - cast(age_r as bigint)) <= 1 then 1 else 0 end"),
    ("height", ["height"], 3,
     "case when cast(height_l as double) is null or cast(height_r as double) is null then -1 "
     "when abs(cast(height_l as double) - cast(height_r as double)) < 0.01 then 2 "
     "when cast(cast(height_l as double) as int) = cast(cast(height_r as double) as int) then 1 else 0 end"),
    # template-shaped Levenshtein-3 over a derived column, null guard on the input column (rewritten)
    ("sn_lev3", ["surname"], 3,
     "case when surname_l is null or surname_r is null then -1 "
     "when upper(trim(surname_l)) = upper(trim(surname_r)) then 2 "
     "when levenshtein(upper(trim(surname_l)), upper(trim(surname_r)))/((length(upper(trim(surname_l))) + "
     "length(upper(trim(surname_r))))/2) <= 0.3 then 1 else 0 end"),
    ("prefix", ["surname"], 2,
     "case when surname_l is null or surname_r is null then -1 "
     "when substr(lower(surname_l), 1, 3) = substr(lower(surname_r), 1, 3) then 1 else 0 end"),
    # Spark built-ins added in round 6: soundex, regular expressions (one with a backslash escape in its literal:
    # the SQL text '\\d' is the regex \d), dates kept as day numbers, datediff as a value test
    ("sx", ["surname"], 2,
     "case when surname_l is null or surname_r is null then -1 when soundex(surname_l) = soundex(surname_r) then 1 "
     "else 0 end"),
    ("rx", ["first_name", "age"], 4,
     "case when first_name_l is null or first_name_r is null then -1 "
     "when regexp_replace(lower(first_name_l), '[^a-z]', '') = regexp_replace(lower(first_name_r), '[^a-z]', '') "
     "then 3 when regexp_extract(first_name_l, '^ *([A-Za-z])(.)', 2) = regexp_extract(first_name_r, '^ *([A-Za-z])(.)', 2) "
     "then 2 when regexp_replace(age_l, '\\\\d', '#') = regexp_replace(age_r, '\\\\d', '#') then 1 else 0 end"),
    ("dd", ["visit"], 4,
     "case when to_date(visit_l) is null or to_date(visit_r) is null then -1 "
     "when to_date(visit_l) = to_date(visit_r) then 3 "
     "when abs(datediff(visit_l, visit_r)) <= 30 then 2 "
     "when datediff(visit_l, visit_r) > 365 or datediff(date_add(visit_l, 7), visit_r) < -100.5 then 1 else 0 end"),
    ("nulls", ["first_name", "age"], 3,
     "case when ifnull(lower(first_name_l), 'zz') = ifnull(lower(first_name_r), 'zz') then 2 "
     "when lower(ifnull(first_name_l, age_l)) = lower(ifnull(first_name_r, age_r)) then 1 else 0 end"),
]


def _settings(link_type="dedupe_only"):
    return {"link_type": link_type, "proportion_of_matches": 0.1, "blocking_rules": ["l.city = r.city"],
            "comparison_columns": [{"custom_name": n, "custom_columns_used": cols, "num_levels": L,
                                    "case_expression": e} for n, cols, L, e in EXPRS],
            "retain_matching_columns": False, "retain_intermediate_calculation_columns": False}


def _oracle(settings, df=None, df_l=None, df_r=None):
    pairs, left, right = orc.block(settings, df=df, df_l=df_l, df_r=df_r)
    cmp_df = orc.comparison_frame(pairs, left, right)
    g = orc.sql_gammas(cmp_df, [c["case_expression"] for c in settings["comparison_columns"]])
    out = pd.DataFrame(g, columns=[f"gamma_{n}" for n, *_ in EXPRS])
    out["unique_id_l"] = cmp_df["unique_id_l"].to_numpy()
    out["unique_id_r"] = cmp_df["unique_id_r"].to_numpy()
    return out.sort_values(["unique_id_l", "unique_id_r"]).reset_index(drop=True)


@pytest.mark.parametrize("link_type", ["dedupe_only", "link_only"])
def test_derived_columns_match_oracle(amd, link_type):
    from splink_amd import add_gammas, block_using_rules, complete_settings_dict
    df = _frame(700, 3)
    st = complete_settings_dict(copy.deepcopy(_settings(link_type)), amd)
    if link_type == "dedupe_only":
        kw = dict(df=df)
    else:
        kw = dict(df_l=df.iloc[:350].reset_index(drop=True), df_r=df.iloc[350:].reset_index(drop=True))
    want = _oracle(st, **kw)
    assert (want.filter(like="gamma_").to_numpy() != -99).all()  # every CASE resolved to a level
    got = add_gammas(block_using_rules(st, amd, **kw), st, amd).toPandas()
    got = got.sort_values(["unique_id_l", "unique_id_r"]).reset_index(drop=True)
    assert len(got) == len(want) > 10000
    for n, *_ in EXPRS:
        g, w = got[f"gamma_{n}"].to_numpy(), want[f"gamma_{n}"].to_numpy()
        bad = np.nonzero(g != w)[0]
        assert len(bad) == 0, (n, len(bad), got.iloc[bad[:3]].to_dict("records"), w[bad[:3]])


def test_derived_jw_column_takes_the_filter(amd):
    """jaro_winkler_sim(lower(a_l), lower(a_r)) names ONE derived column on both sides: the column is
    template-shaped and runs through the filter kernel, with the interpreter giving the same levels."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    df = _frame(3000, 5)
    st = complete_settings_dict(copy.deepcopy(_settings()), amd)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    assert job.ctx.gammas_simple_count() == 2  # fn_jw and sn_lev3: template columns over derived columns
    fast = job.gammas_host()
    job.ctx.gammas_set_simple(0)
    job.gammas(st)
    assert (job.gammas_host() == fast).all()
