"""Host-side encoding of record tables for the device (Arrow-style buffers).

Strings go to the device as UTF-8 + int64 offsets + validity and are decoded there to
UTF-16 code units.  Numbers go as float64 + validity.  A column is uploaded in the form an
operation needs: a numeric column compared with a string function is rendered with Spark's
cast-to-string rules, a string column used numerically is parsed (unparseable -> NULL),
as Spark's implicit casts do.
"""
from __future__ import annotations

import decimal
import math

import numpy as np
import pandas as pd

try:
    import pyarrow as pa
except ImportError:  # pragma: no cover
    pa = None


def is_null_scalar(v) -> bool:
    if v is None:
        return True
    if isinstance(v, float) and math.isnan(v):
        return True
    try:
        return bool(pd.isna(v)) if not isinstance(v, (str, bytes, list, tuple, dict)) else False
    except (TypeError, ValueError):
        return False


def natural_form(series: pd.Series) -> str:
    """'num' for numeric / boolean dtypes, 'str' otherwise."""
    if pd.api.types.is_bool_dtype(series.dtype) or pd.api.types.is_numeric_dtype(series.dtype):
        return "num"
    return "str"


def java_double_str(x: float) -> str:
    """Java Double.toString (what Spark's cast(double as string) prints)."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "-0.0" if math.copysign(1, x) < 0 else "0.0"
    if 1e-3 <= abs(x) < 1e7:
        s = repr(x)
        if "e" in s:
            s = f"{x:.20f}".rstrip("0")
        return s + "0" if s.endswith(".") else (s if "." in s else s + ".0")
    sign, digits, exp = decimal.Decimal(repr(x)).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    e10 = len(digits) - 1 + exp
    mant = ds[0] + "." + (ds[1:] or "0")
    return ("-" if sign else "") + f"{mant}E{e10}"


def spark_str(v) -> str:
    if isinstance(v, str):
        return v
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)):
        return java_double_str(float(v))
    return str(v)


def to_strings(series: pd.Series):
    """Python list of str / None with Spark's cast-to-string rendering."""
    out = []
    for v in series.tolist():
        out.append(None if is_null_scalar(v) else spark_str(v))
    return out


def encode_utf8(series: pd.Series):
    """(offsets int64[n+1], bytes uint8[], valid uint8[n])."""
    n = len(series)
    if pa is not None and series.dtype == object:
        try:
            arr = pa.array(series.to_numpy(), type=pa.large_string(), from_pandas=True)
            return _arrow_buffers(arr, n)
        except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError, UnicodeEncodeError):
            pass
    vals = to_strings(series)
    if pa is not None:
        try:
            arr = pa.array(vals, type=pa.large_string())
            return _arrow_buffers(arr, n)
        except (pa.ArrowInvalid, UnicodeEncodeError):
            pass
    valid = np.array([v is not None for v in vals], dtype=np.uint8)
    enc = [v.encode("utf-8", "surrogatepass") if v is not None else b"" for v in vals]
    offsets = np.zeros(n + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([len(b) for b in enc])
    data = np.frombuffer(b"".join(enc), dtype=np.uint8)
    return offsets, data, valid


def arrow_utf8(series: pd.Series):
    """(offsets int64[n+1], bytes uint8[], valid uint8[n]) of a string column.  Arrow-backed columns
    (pd.ArrowDtype string / large_string, pandas' pyarrow strings) hand over their buffers without a
    per-row pass; object columns of str / None go through pyarrow's converter; anything else is
    rendered with Spark's cast-to-string rules (encode_utf8)."""
    n = len(series)
    if pa is not None:
        arr = getattr(series.array, "_pa_array", None)
        if arr is not None and (pa.types.is_large_string(arr.type) or pa.types.is_string(arr.type)):
            arr = arr.combine_chunks() if isinstance(arr, pa.ChunkedArray) else arr
            if pa.types.is_string(arr.type):
                arr = arr.cast(pa.large_string())
            return _arrow_buffers(arr, n)
    return encode_utf8(series)


def arrow_large_utf8(series: pd.Series):
    """The Arrow large_string array behind a string column (one chunk), or None for other columns."""
    if pa is None:
        return None
    arr = getattr(series.array, "_pa_array", None)
    if arr is None or not (pa.types.is_large_string(arr.type) or pa.types.is_string(arr.type)):
        return None
    arr = arr.combine_chunks() if isinstance(arr, pa.ChunkedArray) else arr
    return arr.cast(pa.large_string()) if pa.types.is_string(arr.type) else arr


def arrow_large_utf8_chunks(series: pd.Series):
    """The chunks of the Arrow string array behind a column, each as large_string (no combine: a chunked
    column is uploaded chunk by chunk), or None for other columns."""
    if pa is None:
        return None
    arr = getattr(series.array, "_pa_array", None)
    if arr is None or not (pa.types.is_large_string(arr.type) or pa.types.is_string(arr.type)):
        return None
    chunks = arr.chunks if isinstance(arr, pa.ChunkedArray) else [arr]
    return [c.cast(pa.large_string()) if pa.types.is_string(c.type) else c for c in chunks]


def arrow_views(arr):
    """Zero-copy numpy views of a large_string array's buffers: (offsets int64[n+1] (any base), data
    uint8, validity bitmap uint8 or None, bit offset of row 0 in it)."""
    n = len(arr)
    bufs = arr.buffers()
    off = np.frombuffer(bufs[1], dtype=np.int64)[arr.offset: arr.offset + n + 1]
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None and bufs[2].size else np.zeros(1, np.uint8)
    bitmap = np.frombuffer(bufs[0], dtype=np.uint8) if (bufs[0] is not None and arr.null_count) else None
    return off, data, bitmap, int(arr.offset)


def numeric_key_bits(series: pd.Series):
    """(int64 values, valid) whose bit patterns are equal iff the numbers are: int64 columns as they
    are, float columns as canonical float64 bits (-0.0 -> 0.0); NaN is NULL."""
    if pd.api.types.is_integer_dtype(series.dtype) and not pd.api.types.is_bool_dtype(series.dtype):
        valid = (~series.isna()).to_numpy()
        vals = series.to_numpy(dtype=np.int64, na_value=0) if hasattr(series, "to_numpy") else series.values
        return np.asarray(vals, dtype=np.int64), valid.astype(np.uint8)
    f = pd.to_numeric(series, errors="coerce").astype(np.float64).to_numpy()
    valid = ~np.isnan(f)
    f = np.where(valid, f, 0.0) + 0.0  # -0.0 + 0.0 == +0.0
    return f.view(np.int64).copy(), valid.astype(np.uint8)


def _arrow_buffers(arr, n):
    arr = arr.combine_chunks() if hasattr(arr, "combine_chunks") else arr
    valid = np.asarray(arr.is_valid()).astype(np.uint8) if arr.null_count else np.ones(n, dtype=np.uint8)
    bufs = arr.buffers()
    off = np.frombuffer(bufs[1], dtype=np.int64)[arr.offset: arr.offset + n + 1].copy()
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
    off0 = off[0]
    data = data[off0: off[-1]].copy()
    off -= off0
    return off, data, valid


def encode_float64(series: pd.Series):
    if natural_form(series) == "num":
        vals = pd.to_numeric(series, errors="coerce").astype(np.float64).to_numpy()
    else:
        vals = pd.to_numeric(pd.Series([None if is_null_scalar(v) else v for v in series.tolist()], dtype=object),
                             errors="coerce").astype(np.float64).to_numpy()
    valid = (~np.isnan(vals)).astype(np.uint8)
    # NaN = NULL (value 0); +-Infinity stay infinite (np.nan_to_num would clamp them to +-DBL_MAX, and then
    # Infinity - Infinity would compare as 0 instead of NaN)
    return np.where(valid.astype(bool), vals, 0.0), valid


def factorize_joint(parts):
    """Shared dense ids (-1 = NULL) for several value arrays, e.g. the l-side and r-side keys."""
    lens = [len(p) for p in parts]
    allv = pd.concat([pd.Series(p, dtype=object) if not isinstance(p, pd.Series) else p.reset_index(drop=True)
                      for p in parts], ignore_index=True)
    codes, uniques = pd.factorize(allv, use_na_sentinel=True)
    out, pos = [], 0
    for n in lens:
        out.append(codes[pos: pos + n].astype(np.int64))
        pos += n
    return out, len(uniques)


def combine_codes(code_lists):
    """Composite ids for tuples of per-term ids; -1 if any term is NULL.  Returns per-part arrays."""
    n_parts = len(code_lists[0])
    acc = [np.zeros(len(code_lists[0][i]), dtype=np.int64) for i in range(n_parts)]
    nulls = [np.zeros(len(code_lists[0][i]), dtype=bool) for i in range(n_parts)]
    for term in code_lists:
        for i in range(n_parts):
            nulls[i] |= term[i] < 0
        card = max(int(max((t.max() if len(t) else -1) for t in term)) + 1, 1)
        for i in range(n_parts):
            acc[i] = acc[i] * card + np.maximum(term[i], 0)
        # re-densify to keep ids small
        dense, _ = factorize_joint([pd.Series(a) for a in acc])
        acc = [d.astype(np.int64) for d in dense]
    return [np.where(nulls[i], -1, acc[i]) for i in range(n_parts)]


def dense_rank(values):
    """Dense rank of the non-NULL values (equal values -> equal rank) in Spark's comparison order,
    and the NULL mask.  Numbers (ints / floats, NULLs aside) compare numerically; anything else by
    its string rendering in code-point order (= Spark's UTF-8 byte order)."""
    vals = list(values)
    nulls = np.array([is_null_scalar(v) for v in vals], dtype=bool)
    present = [v for v, n in zip(vals, nulls) if not n]
    rank = np.zeros(len(vals), dtype=np.int64)
    if present and all(isinstance(v, (int, np.integer, float, np.floating)) and not isinstance(v, (bool, np.bool_))
                       for v in present):
        arr = np.asarray(present, dtype=np.float64 if any(isinstance(v, (float, np.floating)) for v in present)
                         else np.int64)
        _, inv = np.unique(arr, return_inverse=True)
        rank[~nulls] = inv.astype(np.int64)
    elif present:
        keyed = [spark_str(v) for v in present]
        order = {k: i for i, k in enumerate(sorted(set(keyed)))}
        rank[~nulls] = np.array([order[k] for k in keyed], dtype=np.int64)
    return rank, nulls


def dense_rank_array(values: np.ndarray):
    """dense_rank for a numeric numpy array without NULLs (vectorised fast path)."""
    _, inv = np.unique(values, return_inverse=True)
    return inv.astype(np.int64).reshape(-1), np.zeros(len(values), dtype=bool)


def spark_substr(s: str, pos: int, length: int) -> str:
    """Spark UTF8String.substringSQL on code points."""
    n = len(s)
    start = pos - 1 if pos > 0 else (n + pos if pos < 0 else 0)
    end = start + length
    start = max(start, 0)
    if start >= end:
        return ""
    return s[start:min(end, n)]
