"""Settings completion (reference: splink/settings.py:32-231).

`complete_settings_dict` fills defaults, picks each comparison column's default CASE
template (Jaro-Winkler when the session exposes `jaro_winkler_sim`, else equality /
Levenshtein), normalises m / u and assigns `gamma_index`.  Like the reference it mutates
and returns the dict it is given.
"""
import warnings

from .case_statements import (_add_as_gamma_to_case_statement, _check_jaro_registered,
                              _check_no_obvious_problem_with_case_statement, sql_gen_case_smnt_strict_equality_2,
                              sql_gen_case_stmt_levenshtein_3, sql_gen_case_stmt_levenshtein_4,
                              sql_gen_case_stmt_numeric_2, sql_gen_case_stmt_numeric_perc_3,
                              sql_gen_gammas_case_stmt_jaro_2, sql_gen_gammas_case_stmt_jaro_3,
                              sql_gen_gammas_case_stmt_jaro_4)
from .validate import _get_default_value, validate_settings

_DEFAULT_M = {2: [1, 9], 3: [1, 2, 7], 4: [1, 1, 1, 7]}
_DEFAULT_U = {2: [9, 1], 3: [7, 2, 1], 4: [7, 1, 1, 1]}


def _normalise_prob_list(prob_array: list):
    total = sum(prob_array)
    return [p / total for p in prob_array]


def _get_default_case_statements_functions(spark):
    # numeric with 4 levels deliberately maps to the 3-level template (settings.py:42)
    table = {"numeric": {2: sql_gen_case_stmt_numeric_2, 3: sql_gen_case_stmt_numeric_perc_3,
                         4: sql_gen_case_stmt_numeric_perc_3}}
    if _check_jaro_registered(spark):
        table["string"] = {2: sql_gen_gammas_case_stmt_jaro_2, 3: sql_gen_gammas_case_stmt_jaro_3,
                           4: sql_gen_gammas_case_stmt_jaro_4}
    else:
        table["string"] = {2: sql_gen_case_smnt_strict_equality_2, 3: sql_gen_case_stmt_levenshtein_3,
                           4: sql_gen_case_stmt_levenshtein_4}
    return table


def _get_default_case_statement_fn(default_statements, data_type, levels):
    if data_type not in ("string", "numeric"):
        raise ValueError(f"No default case statement available for data type {data_type}, "
                         "please specify a custom case_expression")
    if levels > 4:
        raise ValueError("No default case statement available when levels > 4, "
                         "please specify a custom 'case_expression' within your settings dictionary")
    return default_statements[data_type][levels]


def _get_probabilities(m_or_u, levels):
    if levels > 4:
        raise ValueError("No default m and u probabilities available when levels > 4, "
                         "please specify custom values for 'm_probabilities' and 'u_probabilities' "
                         "within your settings dictionary")
    return _normalise_prob_list((_DEFAULT_M if m_or_u == "m" else _DEFAULT_U)[levels])


def _complete_case_expression(col_settings, spark):
    name = col_settings["custom_name"] if "custom_name" in col_settings else col_settings["col_name"]
    if "case_expression" not in col_settings:
        fn = _get_default_case_statement_fn(_get_default_case_statements_functions(spark),
                                            col_settings["data_type"], col_settings["num_levels"])
        col_settings["case_expression"] = fn(name, name)
    else:
        _check_no_obvious_problem_with_case_statement(col_settings["case_expression"])
        col_settings["case_expression"] = _add_as_gamma_to_case_statement(col_settings["case_expression"], name)


def _complete_probabilities(col_settings: dict, setting_name: str):
    levels = col_settings["num_levels"]
    if setting_name not in col_settings:
        col_settings[setting_name] = _get_probabilities("m" if setting_name == "m_probabilities" else "u", levels)
    elif len(col_settings[setting_name]) != levels:
        raise ValueError(f"Number of {setting_name} provided is not equal to number of levels specified")
    col_settings[setting_name] = _normalise_prob_list(col_settings[setting_name])


def complete_settings_dict(settings_dict: dict, spark):
    """Auto-populate missing settings from the schema defaults (reference settings.py:171-231)."""
    validate_settings(settings_dict)
    for key in ("em_convergence", "unique_id_column_name", "additional_columns_to_retain", "retain_matching_columns",
                "retain_intermediate_calculation_columns", "max_iterations", "proportion_of_matches"):
        if key not in settings_dict:
            settings_dict[key] = _get_default_value(key, is_column_setting=False)
    if "blocking_rules" in settings_dict and len(settings_dict["blocking_rules"]) == 0:
        warnings.warn("You have not specified any blocking rules, meaning all comparisons between the "
                      "input dataset(s) will be generated and blocking will not be used."
                      "For large input datasets, this will generally be computationally intractable "
                      "because it will generate comparisons equal to the number of rows squared.")
    for index, col in enumerate(settings_dict["comparison_columns"]):
        col["gamma_index"] = index
        for key in ("num_levels", "data_type", "term_frequency_adjustments"):
            if key not in col:
                col[key] = _get_default_value(key, is_column_setting=True)
        _complete_case_expression(col, spark)
        _complete_probabilities(col, "m_probabilities")
        _complete_probabilities(col, "u_probabilities")
    return settings_dict
