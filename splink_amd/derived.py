"""Derived columns: Spark built-ins applied to ONE record's columns inside a comparison expression.

The reference splices each completed `case_expression` verbatim into Spark SQL (gammas.py:47, :53), so
any Spark built-in works there; the common hand-written comparisons wrap the `_l` / `_r` operands in a
function of one record -- `jaro_winkler_sim(lower(first_name_l), lower(first_name_r))`,
`trim(x_l) = trim(x_r)`, `cast(age_l as int) = cast(age_r as int)`, `concat(first_name_l, ' ',
surname_l)`.  Such a sub-expression depends on one row of one table only, so it is evaluated ONCE per
row at ingest (Spark semantics below), kept on the device as a column of its own, and every pair reads
it like an input column: the comparison kernels (template filter, exact passes, interpreter) are the
same as for plain columns, and `lower(a_l)` / `lower(a_r)` name one derived column on both sides, so a
template-shaped CASE over it still takes the filter path.

Semantics restated (Apache Spark 2.3/2.4 built-ins, not pinned: SURVEY.md §2.2 N3):
* lower / upper: `UTF8String.toLowerCase / toUpperCase` = Java `String.toLowerCase()` /
  `toUpperCase()`; restated with Python's full Unicode case mapping (identical for ASCII; for other
  text both follow Unicode's SpecialCasing, "parity unpinned" where the Unicode versions differ).
  A number argument is first cast to string (Spark's implicit cast).
* trim / ltrim / rtrim: remove the space character U+0020 only (`UTF8String.trim`), not other
  whitespace.
* concat(a, ...): NULL if any argument is NULL; concat_ws(sep, ...): skips NULL arguments.
* substr(x, pos, len) inside a derived expression: `UTF8String.substringSQL` on code points.
* ifnull / coalesce / nvl(x, literal).
* cast(x as string): strings unchanged, integers in decimal, doubles as Java `Double.toString`.
* cast(x as int / bigint / smallint / tinyint): from a string, Spark 2.4's `UTF8String.toInt/toLong`
  (optional sign, digits, an optional '.' followed only by digits which are truncated; no whitespace;
  anything else or an overflow -> NULL); from a number, truncation toward zero (Scala's `toInt` /
  `toLong`: NaN -> 0, out of range saturates).
* cast(x as double): from a string, Java `Double.parseDouble` (surrounding characters <= U+0020
  trimmed, optional sign, "NaN" / "Infinity", decimal with optional exponent and an optional d / f
  suffix; else NULL).  NaN stays a number in Spark but is NULL in the device's numeric columns (its
  comparisons are false either way, except `IS NULL`): "parity unpinned" for literal NaN strings.
"""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional, Tuple

import numpy as np
import pandas as pd

from . import table as T
from .sqlexpr import Case, Col, Func, Lit

try:
    import pyarrow as pa
    import pyarrow.compute as pc
except ImportError:  # pragma: no cover
    pa = pc = None

STR_FUNCS = ("lower", "lcase", "upper", "ucase", "trim", "ltrim", "rtrim", "concat", "concat_ws")
CAST_TYPES = {"string": "str", "varchar": "str", "int": "int", "integer": "int", "bigint": "long",
              "long": "long", "smallint": "short", "short": "short", "tinyint": "byte", "byte": "byte",
              "double": "double"}
INT_RANGE = {"int": 2 ** 31, "long": 2 ** 63, "short": 2 ** 15, "byte": 2 ** 7}
OPERAND_FUNCS = ("substr", "substring", "ifnull", "coalesce", "nvl")


def is_derived(node) -> bool:
    """A node that makes its operand a derived column (a Spark built-in over one record)."""
    return isinstance(node, Func) and (node.name in STR_FUNCS or node.name == "cast")


def cast_type(node: Func) -> str:
    if len(node.args) != 2 or not isinstance(node.args[1], Lit) or not isinstance(node.args[1].value, str):
        raise ValueError(f"malformed cast: {node}")
    t = node.args[1].value.lower()
    if t not in CAST_TYPES:
        raise ValueError(f"cast(... as {t}) is not supported in a case_expression (supported: "
                         f"{', '.join(sorted(CAST_TYPES))})")
    return CAST_TYPES[t]


def form_of(node, col_form) -> str:
    """Device form ('str' / 'num') of a side-neutral derived expression."""
    if isinstance(node, Func):
        if node.name in STR_FUNCS or node.name in ("substr", "substring"):
            return "str"
        if node.name == "cast":
            return "str" if cast_type(node) == "str" else "num"
        if node.name in ("ifnull", "coalesce", "nvl"):
            return form_of(node.args[0], col_form)
    if isinstance(node, Lit):
        return "str" if isinstance(node.value, str) else "num"
    if isinstance(node, Col):
        return col_form(node.name)
    raise ValueError(f"unsupported expression inside a derived column: {node}")


def render(node) -> str:
    """Canonical text of a side-neutral derived expression (its column name on the device)."""
    if isinstance(node, Col):
        return node.name
    if isinstance(node, Lit):
        if isinstance(node.value, str):
            return "'" + node.value.replace("'", "''") + "'"
        return "null" if node.value is None else repr(node.value)
    if isinstance(node, Func):
        if node.name == "cast":
            return f"cast({render(node.args[0])} as {node.args[1].value.lower()})"
        return f"{node.name}({', '.join(render(a) for a in node.args)})"
    raise ValueError(f"unsupported expression inside a derived column: {node}")


def neutralise(node, column_ref) -> Tuple[object, Optional[int]]:
    """(side-neutral copy of `node`, side): every <col>_l / <col>_r reference becomes the input column,
    all of one side.  column_ref(Col) -> (canonical name, side)."""
    sides = set()

    def walk(n):
        if isinstance(n, Col):
            name, side = column_ref(n)
            sides.add(side)
            return Col(name, "")
        if isinstance(n, Lit):
            return n
        if isinstance(n, Func):
            if n.name == "cast":
                cast_type(n)
                return Func("cast", (walk(n.args[0]), n.args[1]))
            if n.name in STR_FUNCS or n.name in OPERAND_FUNCS:
                return Func(n.name, tuple(walk(a) for a in n.args))
            raise ValueError(f"unsupported function {n.name}() inside {render_any(node)}")
        raise ValueError(f"unsupported expression inside a derived column: {n}")

    out = walk(node)
    if len(sides) > 1:
        raise ValueError(f"{render_any(node)} mixes the _l and _r records: a function of one record is expected")
    return out, (sides.pop() if sides else None)


def render_any(node) -> str:
    try:
        return render(node)
    except ValueError:
        return str(node)


# ---- Spark semantics, per value --------------------------------------------------------------------
# the optional float / double suffix only follows a decimal literal (the third alternative):
# Double.parseDouble("Infinityd") / ("NaNf") throw, so Spark's cast gives NULL
_JAVA_DOUBLE = re.compile(r"[+-]?(NaN|Infinity|((\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)[fFdD]?)\Z")
_JAVA_HEX = re.compile(r"([+-]?)(0[xX](?:[0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP][+-]?\d+)[fFdD]?\Z")


def java_parse_double(s: str) -> Optional[float]:
    """java.lang.Double.parseDouble (what Spark 2.4's cast(string as double) calls); None = NULL."""
    t = s.strip("".join(chr(c) for c in range(0x21)))  # String.trim(): chars <= U+0020
    m = _JAVA_DOUBLE.match(t)
    if not m:
        h = _JAVA_HEX.match(t)  # hexadecimal significand with a binary exponent
        if not h:
            return None
        x = float.fromhex(h.group(2))
        return -x if h.group(1) == "-" else x
    body = t.rstrip("fFdD") if m.group(1) not in ("NaN", "Infinity") else t
    if m.group(1) == "NaN":
        return float("nan")
    if m.group(1) == "Infinity":
        return -math.inf if t.startswith("-") else math.inf
    return float(body)


def spark_string_to_integral(s: str, bound: int) -> Optional[int]:
    """UTF8String.toInt / toLong of Spark 2.4 (cast(string as int / bigint)): optional sign, digits, an
    optional '.' followed only by digits (the fraction is truncated); range [-bound, bound); None = NULL."""
    if not s:
        return None
    i, neg = 0, False
    if s[0] in "+-":
        neg = s[0] == "-"
        i = 1
        if len(s) == 1:
            return None
    digits = ""
    while i < len(s) and s[i] != ".":
        if not ("0" <= s[i] <= "9"):
            return None
        digits += s[i]
        i += 1
    if i < len(s):  # the separator: the fractional part must be well formed
        if not all("0" <= c <= "9" for c in s[i + 1:]):
            return None
    v = int(digits) if digits else 0
    v = -v if neg else v
    return v if -bound <= v < bound else None


def number_to_integral(x, bound: int) -> int:
    """Spark 2.4 non-ANSI Cast of a number to an integral type: Scala Double.toLong for bigint (truncation,
    NaN -> 0, saturating at the long range); for int / smallint / tinyint Double.toInt (saturating at the
    int range) followed by the JVM's wrapping narrowing .toShort / .toByte (Cast.castToShort / castToByte:
    `numeric.toInt(b).toShort`), so cast(40000.0 as smallint) is -25536."""
    if isinstance(x, (int, np.integer)) and not isinstance(x, bool):
        v = int(x)
        # integral narrowing wraps in the JVM (int -> smallint keeps the low bits)
        return ((v + bound) % (2 * bound)) - bound
    x = float(x)
    if math.isnan(x):
        return 0
    sat = 2 ** 63 if bound >= 2 ** 63 else 2 ** 31
    v = sat - 1 if x >= sat else (-sat if x < -sat else int(x))
    return ((v + bound) % (2 * bound)) - bound


def _is_null(v) -> bool:
    return T.is_null_scalar(v)


def _to_str(v):
    return None if _is_null(v) else T.spark_str(v)


def eval_row(node, row) -> object:
    """Value of a side-neutral derived expression for one row (a mapping column -> value); None = NULL."""
    if isinstance(node, Col):
        v = row[node.name]
        return None if _is_null(v) else v
    if isinstance(node, Lit):
        return node.value
    name = node.name
    if name == "cast":
        v = eval_row(node.args[0], row)
        if v is None:
            return None
        t = cast_type(node)
        if t == "str":
            return T.spark_str(v)
        if t == "double":
            return java_parse_double(v) if isinstance(v, str) else float(v)
        bound = INT_RANGE[t]
        return spark_string_to_integral(v, bound) if isinstance(v, str) else number_to_integral(v, bound)
    if name in ("ifnull", "coalesce", "nvl"):
        for a in node.args:
            v = eval_row(a, row)
            if v is not None:
                return v
        return None
    if name in ("substr", "substring"):
        s = _to_str(eval_row(node.args[0], row))
        if s is None:
            return None
        pos = node.args[1].value
        ln = node.args[2].value if len(node.args) > 2 else 2 ** 31 - 1
        return T.spark_substr(s, pos, ln)
    if name == "concat":
        parts = [_to_str(eval_row(a, row)) for a in node.args]
        return None if any(p is None for p in parts) else "".join(parts)
    if name == "concat_ws":
        sep = _to_str(eval_row(node.args[0], row))
        if sep is None:
            return None
        parts = [_to_str(eval_row(a, row)) for a in node.args[1:]]
        return sep.join(p for p in parts if p is not None)
    s = _to_str(eval_row(node.args[0], row))
    if s is None:
        return None
    if name in ("lower", "lcase"):
        return s.lower()
    if name in ("upper", "ucase"):
        return s.upper()
    if name == "trim":
        return s.strip(" ")
    if name == "ltrim":
        return s.lstrip(" ")
    if name == "rtrim":
        return s.rstrip(" ")
    raise ValueError(f"unsupported function {name}()")


# ---- whole columns ------------------------------------------------------------------------------------
def _arrow_str(series: pd.Series):
    """The column as a pyarrow string array when it is one (Arrow-backed or object of str / None)."""
    if pa is None:
        return None
    try:
        if isinstance(series.dtype, pd.ArrowDtype):
            t = series.dtype.pyarrow_dtype
            if not (pa.types.is_string(t) or pa.types.is_large_string(t)):
                return None
            return series.array.__arrow_array__().cast(pa.large_string())
        if series.dtype == object:
            return pa.chunked_array([pa.array(series.tolist(), type=pa.large_string(), from_pandas=True)])
    except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError):
        return None
    return None


def _vector(node, df: pd.DataFrame):
    """Fast path for string-only derived expressions on ASCII text: pyarrow kernels (identical results
    to eval_row there).  None when the expression or the data needs the per-row evaluation."""
    if pc is None:
        return None
    if isinstance(node, Col):
        if T.natural_form(df[node.name]) != "str":
            return None
        return _arrow_str(df[node.name])
    if isinstance(node, Lit):
        return None
    if not isinstance(node, Func):
        return None
    name = node.name
    if name in ("lower", "lcase", "upper", "ucase", "trim", "ltrim", "rtrim") and len(node.args) == 1:
        a = _vector(node.args[0], df)
        if a is None:
            return None
        if name in ("lower", "lcase", "upper", "ucase"):
            if pc.all(pc.string_is_ascii(a)).as_py() is False:
                return None  # non-ASCII text: full Unicode case mapping, per row
            return pc.ascii_lower(a) if name in ("lower", "lcase") else pc.ascii_upper(a)
        f = {"trim": pc.utf8_trim, "ltrim": pc.utf8_ltrim, "rtrim": pc.utf8_rtrim}[name]
        return f(a, characters=" ")
    if name == "concat" and node.args:
        parts = []
        for x in node.args:
            if isinstance(x, Lit) and isinstance(x.value, str):
                parts.append(pa.scalar(x.value, type=pa.large_string()))
            else:
                v = _vector(x, df)
                if v is None:
                    return None
                parts.append(v)
        if all(isinstance(p, pa.Scalar) for p in parts):
            return None
        return pc.binary_join_element_wise(*parts, pa.scalar("", type=pa.large_string()), null_handling="emit_null")
    return None


def evaluate(node, df: pd.DataFrame, form: str) -> pd.Series:
    """The derived column over every row of `df` (input row order), as a device-uploadable series:
    Arrow-backed strings (NULL = null) for form 'str', float64 with NaN = NULL for form 'num'."""
    v = _vector(node, df) if form == "str" else None
    if v is not None:
        return pd.Series(pd.arrays.ArrowExtensionArray(v.cast(pa.large_string())), index=df.index)
    cols = sorted({c.name for c in _columns(node)})
    values = {c: (df[c].to_numpy(dtype=object, na_value=None) if isinstance(df[c].dtype, pd.api.extensions.ExtensionDtype)
                  else df[c].to_numpy()) for c in cols}
    n = len(df)
    out: List[object] = [None] * n
    row: Dict[str, object] = {}
    for i in range(n):
        for c in cols:
            row[c] = values[c][i]
        out[i] = eval_row(node, row)
    if form == "str":
        arr = pa.array([None if x is None else str(x) for x in out], type=pa.large_string()) if pa is not None else None
        if arr is not None:
            return pd.Series(pd.arrays.ArrowExtensionArray(arr), index=df.index)
        return pd.Series(out, dtype=object, index=df.index)
    num = np.array([np.nan if x is None else float(x) for x in out], dtype=np.float64)
    return pd.Series(num, index=df.index)


def _columns(node):
    if isinstance(node, Col):
        yield node
    elif isinstance(node, Func):
        for a in node.args:
            yield from _columns(a)
    elif isinstance(node, Case):  # pragma: no cover - not produced by neutralise
        return
