"""Settings validation and defaults (reference: splink/validate.py, files/settings_jsonschema.json).

The reference validates against a JSON schema with `jsonschema` when it is installed.  The
same constraints are checked here directly (no jsonschema dependency), raising
`ValidationError` (a ValueError) with the reference's message prefix; the defaults are the
schema's defaults (settings_jsonschema.json:38-276).
"""
import copy
import numbers

from .check_types import check_types


class ValidationError(ValueError):
    pass


TOP_DEFAULTS = {
    "proportion_of_matches": 0.3,
    "em_convergence": 0.0001,
    "max_iterations": 25,
    "unique_id_column_name": "unique_id",
    "retain_matching_columns": True,
    "retain_intermediate_calculation_columns": True,
    "blocking_rules": [],
    "additional_columns_to_retain": [],
}
COLUMN_DEFAULTS = {
    "col_name": "",
    "num_levels": 2,
    "data_type": "string",
    "custom_name": "",
    "custom_columns_used": [],
    "term_frequency_adjustments": False,
}
TOP_KEYS = {"$schema", "link_type", *TOP_DEFAULTS, "comparison_columns"}
COLUMN_KEYS = {"col_name", "num_levels", "data_type", "custom_name", "custom_columns_used", "case_expression",
               "m_probabilities", "u_probabilities", "term_frequency_adjustments", "gamma_index"}
LINK_TYPES = ("dedupe_only", "link_only", "link_and_dedupe")

_PREFIX = ("There is an error in your settings dictionary. "
           "To quickly write a valid settings dictionary using autocompelte you might want to try "
           "our online tool https://moj-analytical-services.github.io/splink_settings_editor/ or you can use "
           "the autocomplete features of VS Code - just copy and paste code from the following gist "
           "into VS Code, setting language mode to json, or having saved the file as a .json file\n"
           "https://gist.github.com/RobinL/cfe1152dbd33ae26e05a43d9a0ec85b9"
           "\n\nThe details of the error are as follows:\n")


def _is_num(x):
    return isinstance(x, numbers.Number) and not isinstance(x, bool)


def _is_int(x):
    return isinstance(x, numbers.Integral) and not isinstance(x, bool) or (isinstance(x, float) and x.is_integer())


def _problems(s):
    if not isinstance(s, dict):
        yield "settings must be a dict"
        return
    for k in ("comparison_columns", "link_type"):
        if k not in s:
            yield f"'{k}' is a required property"
    for k in s:
        if k not in TOP_KEYS:
            yield f"Additional properties are not allowed ('{k}' was unexpected)"
    if "link_type" in s and s["link_type"] not in LINK_TYPES:
        yield f"{s['link_type']!r} is not one of {list(LINK_TYPES)}"
    checks = [("proportion_of_matches", 0, 1), ("em_convergence", 1e-12, 0.05), ("max_iterations", 0, 500)]
    for k, lo, hi in checks:
        if k in s:
            v = s[k]
            if not _is_num(v):
                yield f"{k}: {v!r} is not of type 'number'"
            elif not (lo <= v <= hi):
                yield f"{k}: {v!r} is outside [{lo}, {hi}]"
    for k in ("retain_matching_columns", "retain_intermediate_calculation_columns"):
        if k in s and not isinstance(s[k], bool):
            yield f"{k}: {s[k]!r} is not of type 'boolean'"
    if "unique_id_column_name" in s and not isinstance(s["unique_id_column_name"], str):
        yield "unique_id_column_name must be a string"
    for k in ("blocking_rules", "additional_columns_to_retain"):
        if k in s:
            if not isinstance(s[k], list) or not all(isinstance(x, str) for x in s[k]):
                yield f"{k} must be an array of strings"
    cols = s.get("comparison_columns")
    if cols is not None:
        if not isinstance(cols, list) or len(cols) < 1:
            yield "comparison_columns must be a non-empty array"
            return
        for i, c in enumerate(cols):
            if not isinstance(c, dict):
                yield f"comparison_columns[{i}] is not an object"
                continue
            for k in c:
                if k not in COLUMN_KEYS:
                    yield f"comparison_columns[{i}]: Additional properties are not allowed ('{k}' was unexpected)"
            a = "col_name" in c
            b = all(k in c for k in ("custom_name", "custom_columns_used", "case_expression", "num_levels"))
            if a == b:
                yield (f"comparison_columns[{i}] is not valid under exactly one of: "
                       "{col_name} or {custom_name, custom_columns_used, case_expression, num_levels}")
            if "num_levels" in c and (not _is_int(c["num_levels"]) or c["num_levels"] < 2):
                yield f"comparison_columns[{i}].num_levels must be an integer >= 2"
            if "data_type" in c and c["data_type"] not in ("string", "numeric"):
                yield f"comparison_columns[{i}].data_type {c['data_type']!r} is not one of ['string', 'numeric']"
            if "case_expression" in c:
                ce = c["case_expression"]
                if not isinstance(ce, str) or not (("CASE" in ce or "case" in ce) and ("END" in ce or "end" in ce)):
                    yield f"comparison_columns[{i}].case_expression does not match '(CASE|case)' and '(END|end)'"
            for k in ("m_probabilities", "u_probabilities"):
                if k in c and (not isinstance(c[k], list) or len(c[k]) < 2 or not all(_is_num(x) for x in c[k])):
                    yield f"comparison_columns[{i}].{k} must be an array of at least 2 numbers"
            if "custom_columns_used" in c and (not isinstance(c["custom_columns_used"], list)
                                               or len(c["custom_columns_used"]) < 1):
                yield f"comparison_columns[{i}].custom_columns_used must be a non-empty array"
            if "term_frequency_adjustments" in c and not isinstance(c["term_frequency_adjustments"], bool):
                yield f"comparison_columns[{i}].term_frequency_adjustments must be a boolean"
            for k in ("col_name", "custom_name"):
                if k in c and not isinstance(c[k], str):
                    yield f"comparison_columns[{i}].{k} must be a string"


@check_types
def validate_settings(settings_dict: dict):
    """Validate a splink settings dict (reference validate.py:52-89)."""
    errors = list(_problems(settings_dict))
    if errors:
        raise ValidationError(_PREFIX + "\n".join(errors))


def _get_default_value(key, is_column_setting):
    table = COLUMN_DEFAULTS if is_column_setting else TOP_DEFAULTS
    return copy.deepcopy(table[key])
