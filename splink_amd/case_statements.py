"""Comparison-level templates (reference: splink/case_statements.py).

The templates are kept as SQL text because they are part of the settings contract (users
put them in `case_expression`, and saved models carry them).  splink_amd.compiler parses
the text into device programs; the string similarity functions are hand-written gfx950
kernels, so `jaro_winkler_sim` is always available on an AmdSession.
"""
import warnings


def _check_jaro_registered(spark):
    """True when the session exposes `jaro_winkler_sim` (case_statements.py:4-21)."""
    if spark is None:
        return False
    if isinstance(spark, str) and spark == "supress_warnings":
        return False
    for fn in spark.catalog.listFunctions():
        if fn.name == "jaro_winkler_sim":
            return True
    warnings.warn("The jaro_winkler_sim user definined function is not available in Spark "
                  "Or you did not pass 'spark' (the SparkSession) into 'Params' "
                  "Falling back to using levenshtein in the default string comparison functions "
                  "You can import these functions using the scala-udf-similarity-0.0.6.jar provided with Splink")
    return False


def _add_as_gamma_to_case_statement(case_statement: str, gamma_col_name):
    """Lower-case the expression and make its alias `gamma_<name>` (case_statements.py:24-43)."""
    text = case_statement.lower().replace("\n", " ").replace("\r", "").strip()
    if not text.endswith(" end"):
        cut = text.rfind(" end ")
        text = text[: cut + 5]
    return f"{text} as gamma_{gamma_col_name}"


def _check_no_obvious_problem_with_case_statement(case_statement):
    low = case_statement.lower()
    if not all(word in low for word in ("case", "end", "when", "then")):
        raise ValueError("The case expression you provided does not seem to be valid SQL. "
                         f"Expression provided is: '{case_statement}'")


def _finish(body, gamma_col_name):
    return body if gamma_col_name is None else _add_as_gamma_to_case_statement(body, gamma_col_name)


def _null_guard(c):
    return f"when {c}_l is null or {c}_r is null then -1"


def sql_gen_case_smnt_strict_equality_2(col_name, gamma_col_name=None):
    body = (f"case\n    {_null_guard(col_name)}\n    when {col_name}_l = {col_name}_r then 1\n"
            f"    else 0 end as gamma_{gamma_col_name}")
    return _finish(body, gamma_col_name)


def _jaro(col, levels_and_thresholds, gamma_col_name):
    lines = [_null_guard(col)]
    for level, t in levels_and_thresholds:
        lines.append(f"when jaro_winkler_sim({col}_l, {col}_r) > {t} then {level}")
    body = "case\n    " + "\n    ".join(lines) + "\n    else 0 end"
    return _finish(body, gamma_col_name)


def sql_gen_gammas_case_stmt_jaro_2(col_name, gamma_col_name=None, threshold=0.94):
    return _jaro(col_name, [(1, threshold)], gamma_col_name)


def sql_gen_gammas_case_stmt_jaro_3(col_name, gamma_col_name=None, threshold1=0.94, threshold2=0.88):
    return _jaro(col_name, [(2, threshold1), (1, threshold2)], gamma_col_name)


def sql_gen_gammas_case_stmt_jaro_4(col_name, gamma_col_name=None, threshold1=0.94, threshold2=0.88,
                                    threshold3=0.7):
    return _jaro(col_name, [(3, threshold1), (2, threshold2), (1, threshold3)], gamma_col_name)


def _lev_ratio(c):
    return f"levenshtein({c}_l, {c}_r)/((length({c}_l) + length({c}_r))/2)"


def sql_gen_case_stmt_levenshtein_3(col_name, gamma_col_name=None, threshold=0.3):
    body = (f"case\n    {_null_guard(col_name)}\n    when {col_name}_l = {col_name}_r then 2\n"
            f"    when {_lev_ratio(col_name)} <= {threshold}\n    then 1\n    else 0 end")
    return _finish(body, gamma_col_name)


def sql_gen_case_stmt_levenshtein_4(col_name, gamma_col_name=None, threshold1=0.2, threshold2=0.4):
    body = (f"case\n    {_null_guard(col_name)}\n    when {col_name}_l = {col_name}_r then 3\n"
            f"    when {_lev_ratio(col_name)} <= {threshold1}\n    then 2\n"
            f"    when {_lev_ratio(col_name)} <= {threshold2}\n    then 1\n    else 0 end")
    return _finish(body, gamma_col_name)


def _sql_gen_max_of_two_cols(col1, col2):
    return f"\n    case\n    when {col1} > {col2} then {col1}\n    else {col2}\n    end\n    "


def _sql_gen_abs_diff(col1, col2):
    return f"(abs({col1} - {col2}))"


def _numeric(col_name, gamma_col_name, thresholds, perc):
    l, r = f"{col_name}_l", f"{col_name}_r"
    value = _sql_gen_abs_diff(l, r)
    if perc:
        value = f"{value}/abs({_sql_gen_max_of_two_cols(l, r)})"
    lines = [_null_guard(col_name)]
    for level, t in thresholds:
        lines.append(f"when {value} < {t} then {level}")
    body = "case\n    " + "\n    ".join(lines) + "\n    else 0 end"
    return _finish(body, gamma_col_name)


def sql_gen_case_stmt_numeric_2(col_name, gamma_col_name=None):
    return _numeric(col_name, gamma_col_name, [(1, 0.00001)], perc=False)


def sql_gen_case_stmt_numeric_abs_3(col_name, gamma_col_name=None, abs_amount=1, equality_threshold=0.0001):
    return _numeric(col_name, gamma_col_name, [(2, equality_threshold), (1, abs_amount)], perc=False)


def sql_gen_case_stmt_numeric_abs_4(col_name, gamma_col_name=None, abs_amount_low=1, abs_amount_high=10,
                                    equality_threshold=0.0001):
    return _numeric(col_name, gamma_col_name, [(3, equality_threshold), (2, abs_amount_low), (1, abs_amount_high)],
                    perc=False)


def sql_gen_case_stmt_numeric_perc_3(col_name, gamma_col_name=None, per_diff=0.05, equality_threshold=0.0001):
    return _numeric(col_name, gamma_col_name, [(2, equality_threshold), (1, per_diff)], perc=True)


def sql_gen_case_stmt_numeric_perc_4(col_name, gamma_col_name=None, per_diff_low=0.05, per_diff_high=0.10,
                                     equality_threshold=0.0001):
    return _numeric(col_name, gamma_col_name, [(3, equality_threshold), (2, per_diff_low), (1, per_diff_high)],
                    perc=True)


def _sql_gen_get_or_list(col_name, other_name_cols, threshold=0.94):
    # ifnull(.., '1234') keeps a NULL other-name column below the threshold
    terms = [f"jaro_winkler_sim({col_name}_l, ifnull({n}_r, '1234')) > {threshold}" for n in other_name_cols]
    return "(" + " OR ".join(terms) + ")"


def sql_gen_gammas_name_inversion_4(col_name: str, other_name_cols: list, gamma_col_name=None, threshold1=0.94,
                                    threshold2=0.88):
    """Levels: 3 JW > t1; 2 name found inverted in another column; 1 JW > t2; 0 otherwise."""
    body = (f"case\n    {_null_guard(col_name)}\n"
            f"    when jaro_winkler_sim({col_name}_l, {col_name}_r) > {threshold1} then 3\n"
            f"    when {_sql_gen_get_or_list(col_name, other_name_cols, threshold1)} then 2\n"
            f"    when jaro_winkler_sim({col_name}_l, {col_name}_r) > {threshold2} then 1\n"
            f"    else 0 end")
    return _finish(body, gamma_col_name)
