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

STR_FUNCS = ("lower", "lcase", "upper", "ucase", "trim", "ltrim", "rtrim", "concat", "concat_ws", "soundex",
             "regexp_replace", "regexp_extract")
# date functions of one record: their values are dates, kept on the device as numbers (days since 1970-01-01)
DATE_FUNCS = ("to_date", "date_add", "date_sub", "datediff")
CAST_TYPES = {"string": "str", "varchar": "str", "int": "int", "integer": "int", "bigint": "long",
              "long": "long", "smallint": "short", "short": "short", "tinyint": "byte", "byte": "byte",
              "double": "double"}
INT_RANGE = {"int": 2 ** 31, "long": 2 ** 63, "short": 2 ** 15, "byte": 2 ** 7}
OPERAND_FUNCS = ("substr", "substring", "ifnull", "coalesce", "nvl")


def is_derived(node) -> bool:
    """A node that makes its operand a derived column (a Spark built-in over one record)."""
    return isinstance(node, Func) and (node.name in STR_FUNCS or node.name in DATE_FUNCS or node.name == "cast")


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
        if node.name in DATE_FUNCS:
            return "num"
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
            if n.name in STR_FUNCS or n.name in OPERAND_FUNCS or n.name in DATE_FUNCS:
                check_args(n)
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


def check_args(n: Func):
    """Argument shapes of the functions whose later arguments must be literals (checked at compile time, so a
    bad pattern fails as the reference's query would, before any row is evaluated)."""
    if n.name in ("regexp_replace", "regexp_extract"):
        want = (3,) if n.name == "regexp_replace" else (2, 3)
        if len(n.args) not in want or not all(isinstance(a, Lit) and isinstance(a.value, str) for a in n.args[1:2]):
            raise ValueError(f"{n.name}() needs a string-literal pattern")
        pat = java_regex(n.args[1].value)
        if n.name == "regexp_replace":
            if not (isinstance(n.args[2], Lit) and isinstance(n.args[2].value, str)):
                raise ValueError("regexp_replace() needs a string-literal replacement")
            java_replacement(n.args[2].value, pat.groups)
        else:
            idx = n.args[2] if len(n.args) == 3 else Lit(1)  # Spark's default group: 1
            if not (isinstance(idx, Lit) and isinstance(idx.value, int) and not isinstance(idx.value, bool)):
                raise ValueError("regexp_extract() needs a literal group index")
            if not 0 <= idx.value <= pat.groups:  # Matcher.group throws: the reference's query fails
                raise ValueError(f"regexp_extract(): group {idx.value} of a pattern with {pat.groups} groups")
    elif n.name in ("date_add", "date_sub"):
        if len(n.args) != 2 or not (isinstance(n.args[1], Lit) and isinstance(n.args[1].value, int)
                                    and not isinstance(n.args[1].value, bool)):
            raise ValueError(f"{n.name}() needs a literal integer number of days")
    elif n.name == "datediff" and len(n.args) != 2:
        raise ValueError("datediff() takes two dates")
    elif n.name in ("to_date", "soundex") and len(n.args) != 1:
        raise ValueError(f"{n.name}() takes one argument (to_date with a format is not supported)")


# ---- Spark semantics: soundex, regular expressions, dates ---------------------------------------------
_US_ENGLISH = "01230127022455012623017202"  # UTF8String.soundex's code per letter A..Z (H, W: 7 = no separator)


def spark_soundex(s: str) -> str:
    """UTF8String.soundex (Spark 2.4): over the UTF-8 bytes; a first byte that is not an ASCII letter returns the
    string unchanged; letters upper-cased; codes 0 (vowels, Y) separate equal codes, 7 (H, W) are skipped without
    separating; non-letters separate; the first letter then up to three codes, padded with '0'."""
    if s == "":
        return s
    b = s.encode("utf-8")
    first = b[0] - 32 if 97 <= b[0] <= 122 else b[0]
    if not 65 <= first <= 90:
        return s
    sx = [chr(first)]
    last = _US_ENGLISH[first - 65]
    for x in b[1:]:
        x = x - 32 if 97 <= x <= 122 else x
        if not 65 <= x <= 90:
            last = "0"
            continue
        code = _US_ENGLISH[x - 65]
        if code == "7":
            continue
        if code != "0" and code != last:
            sx.append(code)
            if len(sx) > 3:
                break
        last = code
    return "".join(sx).ljust(4, "0")


_REGEX_CACHE: Dict[str, "re.Pattern"] = {}


def java_regex(pattern: str) -> "re.Pattern":
    """A java.util.regex pattern (Spark's regexp_replace / regexp_extract) as a Python pattern.  The common
    subset -- literals, classes, \\d \\w \\s \\b (ASCII in Java: re.ASCII), quantifiers (greedy / lazy), groups,
    alternation, anchors -- means the same in both; constructs Python's re lacks (possessive quantifiers, atomic
    groups, \\p{..} classes, \\Q..\\E) fail to compile here and raise ValueError."""
    p = _REGEX_CACHE.get(pattern)
    if p is None:
        if re.search(r"\\[pPQEGZz]|\(\?>|[*+?}]\+", pattern):
            raise ValueError(f"regular expression {pattern!r} uses a Java construct that is not supported")
        try:
            p = re.compile(pattern, re.ASCII)
        except re.error as e:
            raise ValueError(f"regular expression {pattern!r} does not compile: {e}") from None
        _REGEX_CACHE[pattern] = p
    return p


def java_replacement(rep: str, groups: int):
    """Matcher.appendReplacement's replacement string as a list of literal strings and group numbers: \\x is the
    character x, $n a group (the longest group number that exists, as Java reads it), a '$' or '\\' at the end
    is an error."""
    parts: List[object] = []
    lit = []
    i = 0
    while i < len(rep):
        c = rep[i]
        if c == "\\":
            if i + 1 >= len(rep):
                raise ValueError("regexp_replace(): character to be escaped is missing")
            lit.append(rep[i + 1])
            i += 2
        elif c == "$":
            if i + 1 >= len(rep) or not rep[i + 1].isdigit():
                raise ValueError("regexp_replace(): illegal group reference")
            g = int(rep[i + 1])
            if g > groups:
                raise ValueError(f"regexp_replace(): no group {g}")
            i += 2
            while i < len(rep) and rep[i].isdigit() and g * 10 + int(rep[i]) <= groups:
                g = g * 10 + int(rep[i])
                i += 1
            if lit:
                parts.append("".join(lit))
                lit = []
            parts.append(g)
        else:
            lit.append(c)
            i += 1
    if lit:
        parts.append("".join(lit))
    return parts


def spark_regexp_replace(s: str, pattern: str, rep: str) -> str:
    p = java_regex(pattern)
    parts = java_replacement(rep, p.groups)
    return p.sub(lambda m: "".join(x if isinstance(x, str) else (m.group(x) or "") for x in parts), s)


def spark_regexp_extract(s: str, pattern: str, idx: int = 1) -> str:
    """RegExpExtract: the group of the first match; '' without a match or for a group that did not take part."""
    m = java_regex(pattern).search(s)
    return "" if m is None else (m.group(idx) or "")


class Day(int):
    """A date value inside a derived expression: days since 1970-01-01 (rendered 'yyyy-MM-dd' as a string)."""


_MONTH31 = (1, 3, 5, 7, 8, 10, 12)


def _leap(y: int) -> bool:
    return y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)


def epoch_day(y: int, m: int, d: int) -> int:
    """Days since 1970-01-01 of a date as java.util.GregorianCalendar (GMT) reads it: Gregorian from 1582-10-15,
    Julian before (the reference's Spark 2.4 uses the hybrid calendar; parity unpinned before 1582)."""
    if (y, m, d) >= (1582, 10, 15):
        a = (14 - m) // 12
        yy, mm = y + 4800 - a, m + 12 * a - 3
        jdn = d + (153 * mm + 2) // 5 + 365 * yy + yy // 4 - yy // 100 + yy // 400 - 32045
    else:
        a = (14 - m) // 12
        yy, mm = y + 4800 - a, m + 12 * a - 3
        jdn = d + (153 * mm + 2) // 5 + 365 * yy + yy // 4 - 32083
    return jdn - 2440588


def day_to_string(day: int) -> str:
    """'yyyy-MM-dd' of a day number (Gregorian from 1582-10-15, Julian before, as epoch_day)."""
    jdn = int(day) + 2440588
    if jdn >= 2299161:  # 1582-10-15
        a = jdn + 32044
        b = (4 * a + 3) // 146097
        c = a - 146097 * b // 4
    else:
        b = 0
        c = jdn + 32082
    d_ = (4 * c + 3) // 1461
    e = c - 1461 * d_ // 4
    m_ = (5 * e + 2) // 153
    day_ = e - (153 * m_ + 2) // 5 + 1
    month = m_ + 3 - 12 * (m_ // 10)
    year = 100 * b + d_ - 4800 + m_ // 10
    return f"{year:04d}-{month:02d}-{day_:02d}"


def spark_string_to_date(s: str) -> Optional[int]:
    """DateTimeUtils.stringToDate (Spark 2.4) as days since 1970-01-01; None = NULL.  Spaces trimmed; 'yyyy',
    'yyyy-[m]m', 'yyyy-[m]m-[d]d', optionally followed by ' ' or 'T' and anything; the year exactly four digits;
    missing month / day are 1; an impossible date is NULL."""
    b = s.strip(" ").encode("utf-8")
    seg = [1, 1, 1]
    i = cur = j = 0
    while j < len(b) and b[j] not in (0x20, 0x54):  # ' ', 'T'
        c = b[j]
        if i < 2 and c == 0x2D:  # '-'
            if i == 0 and j != 4:
                return None
            seg[i] = cur
            cur = 0
            i += 1
        elif 0x30 <= c <= 0x39:
            cur = cur * 10 + (c - 0x30)
        else:
            return None
        j += 1
    if i == 0 and j != 4:
        return None
    seg[i] = cur
    y, m, d = seg
    if y < 0 or y > 9999 or m < 1 or m > 12 or d < 1 or d > 31:
        return None
    if m == 2 and d > (29 if _leap(y) else 28):
        return None
    if m not in _MONTH31 and d > 30:
        return None
    return epoch_day(y, m, d)


def to_day(v) -> Optional[int]:
    """A value as a date (days since 1970-01-01): a date value, a string (stringToDate), a datetime / date
    object; numbers are not dates (NULL)."""
    if v is None:
        return None
    if isinstance(v, Day):
        return int(v)
    if isinstance(v, str):
        return spark_string_to_date(v)
    if hasattr(v, "year") and hasattr(v, "month") and hasattr(v, "day"):
        return epoch_day(int(v.year), int(v.month), int(v.day))
    return None


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
    if isinstance(v, Day):
        return day_to_string(v)
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
            return _to_str(v)
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
    if name in DATE_FUNCS:
        days = to_day(eval_row(node.args[0], row))
        if days is None:
            return None
        if name == "to_date":
            return Day(days)
        if name in ("date_add", "date_sub"):
            k = node.args[1].value
            return Day(days + (k if name == "date_add" else -k))
        other = to_day(eval_row(node.args[1], row))
        return None if other is None else days - other  # datediff(end, start): an integer
    if name in ("regexp_replace", "regexp_extract"):
        s = _to_str(eval_row(node.args[0], row))
        if s is None:
            return None
        if name == "regexp_replace":
            return spark_regexp_replace(s, node.args[1].value, node.args[2].value)
        return spark_regexp_extract(s, node.args[1].value, node.args[2].value if len(node.args) > 2 else 1)
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
    if name == "soundex":
        return spark_soundex(s)
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
    num = np.array([np.nan if x is None else float(x) for x in out], dtype=np.float64)  # a date: its day number
    return pd.Series(num, index=df.index)


def _columns(node):
    if isinstance(node, Col):
        yield node
    elif isinstance(node, Func):
        for a in node.args:
            yield from _columns(a)
    elif isinstance(node, Case):  # pragma: no cover - not produced by neutralise
        return
