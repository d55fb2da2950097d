"""CPU oracle for splink's comparison + EM hot path.

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  The product never imports it.

Two layers, both restating the reference's semantics independently of the
product code:

* `liboracle.so` (splink_oracle.c): Jaro-Winkler (commons-text 1.4, UTF-16
  units), Levenshtein (Spark, code points), the standard comparison templates,
  the E-step and the M-step sufficient statistics, OpenMP-parallel.
* this module: the reference's SQL semantics for blocking and arbitrary CASE
  expressions, executed by sqlite with the C functions registered as UDFs
  (blocking.py:95-160,219-268; gammas.py:65-89), and the EM driver loop
  (iterate.py:37-63, maximisation_step.py:16-117, params.py:248-336).

Pinned by the reference-generated fixtures in tests/golden/ (see
tests/test_oracle_golden.py).
"""
from __future__ import annotations

import ctypes
import datetime as _dt
import os
import re
import sqlite3
import subprocess

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, "liboracle.so")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return _LIB_PATH


def _lib():
    global _LIB
    try:
        return _LIB
    except NameError:
        pass
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    lib.orc_jaro_winkler_u16.restype = ctypes.c_double
    lib.orc_jaro_winkler_u16.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    lib.orc_levenshtein_u32.restype = ctypes.c_int64
    lib.orc_levenshtein_u32.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    lib.orc_gammas.restype = ctypes.c_int
    lib.orc_em_stats.restype = ctypes.c_int
    lib.orc_score.restype = None
    lib.orc_log_likelihood.restype = None
    lib.orc_em_stats_weighted.restype = ctypes.c_int
    lib.orc_pattern_codes.restype = None
    _LIB = lib
    return lib


def _u16(s: str) -> np.ndarray:
    return np.frombuffer(s.encode("utf-16-le", "surrogatepass"), dtype=np.uint16)


def _u32(s: str) -> np.ndarray:
    return np.array([ord(c) for c in s], dtype=np.uint32)


def jaro_winkler(a, b):
    if a is None or b is None:
        return None
    x, y = _u16(a), _u16(b)
    return _lib().orc_jaro_winkler_u16(x.ctypes.data, len(x), y.ctypes.data, len(y))


def levenshtein(a, b):
    if a is None or b is None:
        return None
    x, y = _u32(a), _u32(b)
    return int(_lib().orc_levenshtein_u32(x.ctypes.data, len(x), y.ctypes.data, len(y)))


# ------------------------------------------------------------------------------------
# string columns for the bulk template path
# ------------------------------------------------------------------------------------
class _StrColC(ctypes.Structure):
    _fields_ = [("u16", ctypes.c_void_p), ("off16", ctypes.c_void_p), ("u32", ctypes.c_void_p),
                ("off32", ctypes.c_void_p), ("valid", ctypes.c_void_p)]


class StrCol:
    """A string column encoded as UTF-16 units and code points (the JW / Levenshtein alphabets).

    Built with whole-column codecs (one join + encode per alphabet), so a 1M-row column takes
    well under a second; lone surrogates pass through as in a Java String."""

    def __init__(self, values):
        vals = [None if (v is None or v is pd.NA or (isinstance(v, float) and np.isnan(v))) else str(v)
                for v in values]
        n = len(vals)
        self.valid = np.array([v is not None for v in vals], dtype=np.uint8)
        strs = [v if v is not None else "" for v in vals]
        len32 = np.fromiter((len(v) for v in strs), dtype=np.int64, count=n)
        joined = "".join(strs)
        u32 = np.frombuffer(joined.encode("utf-32-le", "surrogatepass"), dtype=np.uint32)
        self.off32 = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(len32, out=self.off32[1:])
        supp = (u32 >= 0x10000).astype(np.int64)
        csupp = np.zeros(len(u32) + 1, dtype=np.int64)
        np.cumsum(supp, out=csupp[1:])
        self.off16 = self.off32 + csupp[self.off32]
        self.u16 = np.concatenate([np.frombuffer(joined.encode("utf-16-le", "surrogatepass"), dtype=np.uint16),
                                   np.zeros(1, np.uint16)])
        self.u32 = np.concatenate([u32, np.zeros(1, np.uint32)])
        assert self.off16[-1] == len(self.u16) - 1
        self.c = _StrColC(self.u16.ctypes.data, self.off16.ctypes.data, self.u32.ctypes.data,
                          self.off32.ctypes.data, self.valid.ctypes.data)


KIND = {"eq": 0, "jw": 1, "lev": 2}


def template_gammas(specs, cols_l, cols_r, pl, pr):
    """gammas (int8 [P, K]) for standard templates.  specs: [(kind, num_levels, thresholds)]."""
    K = len(specs)
    kinds = np.array([KIND[s[0]] for s in specs], dtype=np.int32)
    nlev = np.array([s[1] for s in specs], dtype=np.int32)
    thr = np.zeros((K, 3), dtype=np.float64)
    for k, s in enumerate(specs):
        thr[k, :len(s[2])] = s[2]
    arr_l = (_StrColC * K)(*[c.c for c in cols_l])
    arr_r = arr_l if cols_r is cols_l else (_StrColC * K)(*[c.c for c in cols_r])
    pl = np.ascontiguousarray(pl, dtype=np.int32)
    pr = np.ascontiguousarray(pr, dtype=np.int32)
    out = np.empty((len(pl), K), dtype=np.int8)
    _lib().orc_gammas(ctypes.c_int(K), kinds.ctypes.data_as(ctypes.c_void_p), nlev.ctypes.data_as(ctypes.c_void_p),
                      thr.ctypes.data_as(ctypes.c_void_p), ctypes.cast(arr_l, ctypes.c_void_p),
                      ctypes.cast(arr_r, ctypes.c_void_p), ctypes.c_int64(len(pl)),
                      pl.ctypes.data_as(ctypes.c_void_p), pr.ctypes.data_as(ctypes.c_void_p),
                      out.ctypes.data_as(ctypes.c_void_p))
    return out


# ------------------------------------------------------------------------------------
# E / M with Spark numeric semantics
# ------------------------------------------------------------------------------------
def quantise(p):
    """`cast({p:.35f} as double)` (expectation_step.py:212)."""
    return float(f"{p:.35f}")


def f32(x):
    """`cast(... as float)` (maximisation_step.py:19, 68-69)."""
    return None if x is None else float(np.float32(x))


def em_stats(gam, nlev, lam, m, u):
    """Sufficient statistics of one E+M pass (layout documented in splink_oracle.c)."""
    gam = np.ascontiguousarray(gam, dtype=np.int8)
    nlev = np.ascontiguousarray(nlev, dtype=np.int32)
    K = len(nlev)
    mq = np.array([quantise(x) for row in m for x in row], dtype=np.float64)
    uq = np.array([quantise(x) for row in u for x in row], dtype=np.float64)
    n_stats = 3 + 4 * int(np.sum(nlev + 1))
    out = np.zeros(n_stats, dtype=np.float64)
    lamd = float(repr(lam))
    one_minus = float(repr(1 - lam))
    _lib().orc_em_stats(ctypes.c_int(K), nlev.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(gam.shape[0]),
                        gam.ctypes.data_as(ctypes.c_void_p), ctypes.c_double(lamd), ctypes.c_double(one_minus),
                        mq.ctypes.data_as(ctypes.c_void_p), uq.ctypes.data_as(ctypes.c_void_p),
                        out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(0))
    return out


def score(gam, nlev, lam, m, u):
    """Final E-step: match_probability per pair, NaN where the reference yields NULL."""
    gam = np.ascontiguousarray(gam, dtype=np.int8)
    nlev = np.ascontiguousarray(nlev, dtype=np.int32)
    mq = np.array([quantise(x) for row in m for x in row], dtype=np.float64)
    uq = np.array([quantise(x) for row in u for x in row], dtype=np.float64)
    out = np.empty(gam.shape[0], dtype=np.float64)
    _lib().orc_score(ctypes.c_int(len(nlev)), nlev.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(gam.shape[0]),
                     gam.ctypes.data_as(ctypes.c_void_p), ctypes.c_double(float(repr(lam))),
                     ctypes.c_double(float(repr(1 - lam))), mq.ctypes.data_as(ctypes.c_void_p),
                     uq.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p))
    return out


def log_likelihood(gam, nlev, lam, m, u):
    """get_overall_log_likelihood (expectation_step.py:224-272): Σ ln(λΠm + (1-λ)Πu) over the pairs,
    None when every term is NULL (Spark's sum of no values)."""
    gam = np.ascontiguousarray(gam, dtype=np.int8)
    nlev = np.ascontiguousarray(nlev, dtype=np.int32)
    mq = np.array([quantise(x) for row in m for x in row], dtype=np.float64)
    uq = np.array([quantise(x) for row in u for x in row], dtype=np.float64)
    out = np.zeros(2, dtype=np.float64)
    _lib().orc_log_likelihood(ctypes.c_int(len(nlev)), nlev.ctypes.data_as(ctypes.c_void_p),
                              ctypes.c_int64(gam.shape[0]), gam.ctypes.data_as(ctypes.c_void_p),
                              ctypes.c_double(float(repr(lam))), ctypes.c_double(float(repr(1 - lam))),
                              mq.ctypes.data_as(ctypes.c_void_p), uq.ctypes.data_as(ctypes.c_void_p),
                              out.ctypes.data_as(ctypes.c_void_p))
    return float(out[0]) if out[1] > 0 else None


def m_step(stats, nlev):
    """New λ and π from the statistics, with Spark's NULL / float32 semantics
    (maximisation_step.py:16-90; params.py:248-274 drops level -1, absent levels -> 0)."""
    S, rows, nn = stats[0], stats[1], stats[2]
    lam = f32(S / rows) if (nn > 0 and rows > 0) else None
    m_new, u_new = [], []
    off = 0
    for L in nlev:
        slots = stats[3 + 4 * off: 3 + 4 * (off + L + 1)].reshape(L + 1, 4)
        off += L + 1
        valid = slots[1:]
        den_ok = valid[:, 1].sum() > 0
        den_m, den_u = valid[:, 2].sum(), valid[:, 3].sum()
        mk, uk = [], []
        for v in range(L):
            r, nnv, sm, su = slots[v + 1]
            if r == 0:
                mk.append(0)
                uk.append(0)
                continue
            if nnv == 0 or not den_ok:
                mk.append(None)
                uk.append(None)
                continue
            mk.append(f32(sm / den_m) if den_m != 0 else None)
            uk.append(f32(su / den_u) if den_u != 0 else None)
        m_new.append(mk)
        u_new.append(uk)
    return lam, m_new, u_new


def pattern_codes(gam, nlev, hist=None, want_codes=True):
    """Mixed-radix pattern index per comparison vector (Σ (γ_k + 1) Π_{j<k} (L_j + 1)); counts are ADDED
    to `hist` (int64 [Π (L_k + 1)]) when given, so chunks of a large pair set accumulate."""
    gam = np.ascontiguousarray(gam, dtype=np.int8)
    nlev = np.ascontiguousarray(nlev, dtype=np.int32)
    n_pat = int(np.prod(nlev.astype(np.int64) + 1))
    out = np.empty(gam.shape[0], dtype=np.int32) if want_codes else None
    _lib().orc_pattern_codes(ctypes.c_int(len(nlev)), nlev.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(gam.shape[0]),
                             gam.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(n_pat),
                             None if out is None else out.ctypes.data_as(ctypes.c_void_p),
                             None if hist is None else hist.ctypes.data_as(ctypes.c_void_p))
    return out


def patterns_of(nlev):
    """Every comparison vector of the pattern space, row p = the vector whose pattern index is p."""
    nlev = [int(x) for x in nlev]
    n_pat = int(np.prod([L + 1 for L in nlev]))
    idx = np.arange(n_pat, dtype=np.int64)
    cols = []
    for L in nlev:
        cols.append((idx % (L + 1)) - 1)
        idx //= L + 1
    return np.stack(cols, axis=1).astype(np.int8)


def em_stats_hist(hist, nlev, lam, m, u):
    """em_stats over a pattern histogram (distinct comparison vectors with their pair counts)."""
    nlev = np.ascontiguousarray(nlev, dtype=np.int32)
    hist = np.asarray(hist, dtype=np.int64)
    pats = patterns_of(nlev)
    nz = np.nonzero(hist)[0]
    g = np.ascontiguousarray(pats[nz])
    w = np.ascontiguousarray(hist[nz])
    mq = np.array([quantise(x) for row in m for x in row], dtype=np.float64)
    uq = np.array([quantise(x) for row in u for x in row], dtype=np.float64)
    out = np.zeros(3 + 4 * int(np.sum(nlev + 1)), dtype=np.float64)
    _lib().orc_em_stats_weighted(ctypes.c_int(len(nlev)), nlev.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(len(nz)),
                                 g.ctypes.data_as(ctypes.c_void_p), w.ctypes.data_as(ctypes.c_void_p),
                                 ctypes.c_double(float(repr(lam))), ctypes.c_double(float(repr(1 - lam))),
                                 mq.ctypes.data_as(ctypes.c_void_p), uq.ctypes.data_as(ctypes.c_void_p),
                                 out.ctypes.data_as(ctypes.c_void_p))
    return out


def em_iterate_hist(hist, nlev, lam, m, u, max_iterations, em_convergence):
    """em_iterate on a pattern histogram; the final mp is returned per pattern index (NaN = NULL)."""
    history = []
    for _ in range(max_iterations):
        stats = em_stats_hist(hist, nlev, lam, m, u)
        new_lam, new_m, new_u = m_step(stats, nlev)
        old = [x for row in m for x in row] + [x for row in u for x in row]
        new = [x for row in new_m for x in row] + [x for row in new_u for x in row]
        lam, m, u = new_lam, new_m, new_u
        history.append((lam, [list(r) for r in m], [list(r) for r in u]))
        if all(abs(a - b) < em_convergence for a, b in zip(new, old)):  # params.py:316-336
            break
    return history, score(patterns_of(nlev), nlev, lam, m, u)


def em_iterate(gam, nlev, lam, m, u, max_iterations, em_convergence):
    """iterate.py:37-63 on a gamma matrix; returns (history of (λ, m, u) after each M-step, final mp)."""
    history = []
    for _ in range(max_iterations):
        stats = em_stats(gam, nlev, lam, m, u)
        new_lam, new_m, new_u = m_step(stats, nlev)
        old = [x for row in m for x in row] + [x for row in u for x in row]
        new = [x for row in new_m for x in row] + [x for row in new_u for x in row]
        lam, m, u = new_lam, new_m, new_u
        history.append((lam, [list(r) for r in m], [list(r) for r in u]))
        if all(abs(a - b) < em_convergence for a, b in zip(new, old)):  # params.py:316-336
            break
    return history, score(gam, nlev, lam, m, u)


# ------------------------------------------------------------------------------------
# Reference SQL semantics through sqlite (small inputs)
# ------------------------------------------------------------------------------------
def _length(s):
    return None if s is None else float(len(s))


def _lev(a, b):
    v = levenshtein(a, b)
    return None if v is None else float(v)


# Spark built-ins over one record (Apache Spark 2.3/2.4, unpinned: SURVEY.md §2.2 N3), restated for sqlite,
# whose own lower / upper are ASCII-only, whose concat() skips NULLs and whose CAST accepts '12abc' as 12.
def _s(v):
    """Spark's implicit cast to string of a sqlite value (strings and integers only in the tests)."""
    if v is None or isinstance(v, str):
        return v
    if isinstance(v, int):
        return str(v)
    raise ValueError(f"oracle: no Java rendering for {v!r}")


def _spark_lower(v):
    v = _s(v)
    return None if v is None else v.lower()  # Java String.toLowerCase; non-ASCII: parity unpinned


def _spark_upper(v):
    v = _s(v)
    return None if v is None else v.upper()


def _spark_trim(v, how="both"):
    v = _s(v)
    if v is None:
        return None
    while how in ("both", "left") and v.startswith(" "):  # UTF8String.trim: U+0020 only
        v = v[1:]
    while how in ("both", "right") and v.endswith(" "):
        v = v[:-1]
    return v


def _spark_concat(*args):
    parts = [_s(a) for a in args]
    return None if any(p is None for p in parts) else "".join(parts)


def _spark_concat_ws(sep, *args):
    if sep is None:
        return None
    return _s(sep).join(p for p in (_s(a) for a in args) if p is not None)


def _spark_to_integral(v, bits):
    """cast(x as int / bigint / smallint / tinyint) (UTF8String.toInt / toLong, Spark 2.4).  A number:
    Cast.castToInt / castToShort / castToByte take `numeric.toInt(b)` (a double saturates at the int range,
    NaN -> 0; bigint: Double.toLong at the long range) and narrow with the JVM's wrapping .toShort / .toByte;
    an integral value narrows by wrapping.  (Restated from Spark 2.4's Cast.scala, which is not in
    /root/reference: parity unpinned for out-of-range numbers.)"""
    if v is None:
        return None
    lim = 2 ** (bits - 1)
    if isinstance(v, float):
        if v != v:
            return 0
        sat = 2 ** 63 if bits == 64 else 2 ** 31
        x = sat - 1 if v >= sat else (-sat if v < -sat else int(v))
        return ((x + lim) % (2 * lim)) - lim
    if isinstance(v, int):
        return ((v + lim) % (2 * lim)) - lim
    m = re.fullmatch(r"([+-]?)([0-9]*)(\.[0-9]*)?", v)
    if not m or v in ("", "+", "-"):
        return None
    x = int(m.group(2) or "0") * (-1 if m.group(1) == "-" else 1)
    lim = 2 ** (bits - 1)
    return x if -lim <= x < lim else None


def _spark_to_double(v):
    """cast(x as double): java.lang.Double.parseDouble of the string (Spark 2.4); NULL when it throws."""
    if v is None or isinstance(v, (int, float)):
        return None if v is None else float(v)
    t = v.strip("".join(chr(c) for c in range(33)))
    m = re.fullmatch(r"([+-]?)(NaN|Infinity|(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?)[fFdD]?", t)
    if not m:
        h = re.fullmatch(r"([+-]?)0[xX]([0-9a-fA-F]*)\.?([0-9a-fA-F]*)[pP]([+-]?[0-9]+)[fFdD]?", t)
        if not h or not (h.group(2) or h.group(3)):
            return None
        x = (int((h.group(2) or "0") + h.group(3), 16) / 16 ** len(h.group(3))) * 2.0 ** int(h.group(4))
        return -x if h.group(1) == "-" else x
    if m.group(2) in ("NaN", "Infinity") and t[-1] in "fFdD":
        return None
    if m.group(2) == "NaN":
        return None  # the device keeps NaN as NULL in numeric columns: parity unpinned for it
    body = m.group(2)
    x = float("inf") if body == "Infinity" else float(body)
    return -x if m.group(1) == "-" else x


_CASTS = {"int": lambda v: _spark_to_integral(v, 32), "integer": lambda v: _spark_to_integral(v, 32),
          "bigint": lambda v: _spark_to_integral(v, 64), "long": lambda v: _spark_to_integral(v, 64),
          "smallint": lambda v: _spark_to_integral(v, 16), "tinyint": lambda v: _spark_to_integral(v, 8),
          "double": _spark_to_double, "string": _s}


def spark_literals(expr):
    """Single-quoted string literals re-quoted for sqlite with the value Spark's parser reads (backslash escapes:
    ParserUtils.unescapeSQLString -- \\0 \\b \\n \\r \\t \\Z \\\\ \\' \\", \\% / \\_ keep the backslash, any other escaped
    character is itself, \\uXXXX, octal \\[01][0-7][0-7]); '' stays one quote."""
    esc = {"0": "\0", "b": "\b", "n": "\n", "r": "\r", "t": "\t", "Z": "\x1a", "%": "\\%", "_": "\\_"}

    def value(body):
        out, i = "", 0
        while i < len(body):
            c = body[i]
            if c == "'":  # '' (the tokenizer only lets doubled quotes through)
                out += "'"
                i += 2
            elif c == "\\" and i + 1 < len(body):
                if body[i + 1] == "u" and re.fullmatch(r"[0-9a-fA-F]{4}", body[i + 2:i + 6] or "") and i + 5 < len(body):
                    out += chr(int(body[i + 2:i + 6], 16))
                    i += 6
                elif re.fullmatch(r"[01][0-7][0-7]", body[i + 1:i + 4]) and i + 3 < len(body):
                    out += chr(int(body[i + 1:i + 4], 8))
                    i += 4
                else:
                    out += esc.get(body[i + 1], body[i + 1])
                    i += 2
            else:
                out += c
                i += 1
        return out

    return re.sub(r"'((?:[^'\\]|\\.|'')*)'", lambda m: "'" + value(m.group(1)).replace("'", "''") + "'", expr)


def rewrite_casts(expr):
    """CAST(x AS t) -> spark_cast_t(x) (sqlite's CAST has other semantics)."""
    out, i = [], 0
    low = expr.lower()
    while True:
        j = low.find("cast(", i)
        if j < 0 or (j > 0 and (low[j - 1].isalnum() or low[j - 1] == "_")):
            if j < 0:
                out.append(expr[i:])
                return "".join(out)
            out.append(expr[i:j + 5])
            i = j + 5
            continue
        out.append(expr[i:j])
        depth, k, as_at = 0, j + 4, -1
        while True:
            c = expr[k]
            if c == "(":
                depth += 1
            elif c == ")":
                depth -= 1
                if depth == 0:
                    break
            elif c == "'":
                k = expr.index("'", k + 1)
            elif depth == 1 and low.startswith(" as ", k):
                as_at = k
            k += 1
        inner, typ = expr[j + 5:as_at], expr[as_at + 4:k].strip().lower()
        out.append(f"spark_cast_{typ}({rewrite_casts(inner)})")
        i = k + 1


# ---- soundex, regular expressions, dates (Spark 2.4 built-ins; not in /root/reference: parity unpinned) -----------
_SOUNDEX_CODES = dict(zip("ABCDEFGHIJKLMNOPQRSTUVWXYZ", "01230127022455012623017202"))


def _spark_soundex(v):
    """UTF8String.soundex: first byte an ASCII letter (else the input), then up to three codes of the later letters;
    vowels and Y (0) and non-letters separate repeated codes, H and W (7) do not."""
    if v is None:
        return None
    v = _s(v)
    if not v:
        return v
    raw = v.encode("utf-8")
    head = chr(raw[0]).upper() if raw[0] < 128 else ""
    if head not in _SOUNDEX_CODES:
        return v
    out, prev = head, _SOUNDEX_CODES[head]
    for byte in raw[1:]:
        ch = chr(byte).upper() if byte < 128 else ""
        code = _SOUNDEX_CODES.get(ch)
        if code is None:
            prev = "0"
        elif code != "7":
            if code not in ("0", prev):
                out += code
            prev = code
        if len(out) == 4:
            break
    return (out + "000")[:4]


def _java_rep(rep, m):
    """Matcher.appendReplacement: \\c -> c, $g -> group g (digits taken while the group exists)."""
    res, i = [], 0
    while i < len(rep):
        if rep[i] == "\\":
            res.append(rep[i + 1])
            i += 2
        elif rep[i] == "$":
            j = i + 2
            while j < len(rep) and rep[j].isdigit() and int(rep[i + 1:j + 1]) <= m.re.groups:
                j += 1
            res.append(m.group(int(rep[i + 1:j])) or "")
            i = j
        else:
            res.append(rep[i])
            i += 1
    return "".join(res)


def _spark_regexp_replace(v, pat, rep):
    if v is None or pat is None or rep is None:
        return None
    return re.compile(pat, re.ASCII).sub(lambda m: _java_rep(rep, m), _s(v))


def _spark_regexp_extract(v, pat, idx=1):
    if v is None or pat is None:
        return None
    m = re.compile(pat, re.ASCII).search(_s(v))
    return (m.group(int(idx)) or "") if m else ""


_DATE = re.compile(r"(\d{4})(?:-(\d*)(?:-(\d*))?)?(?:[ T].*)?", re.DOTALL)


def _days(v):
    """DateTimeUtils.stringToDate of a string as days since 1970-01-01 (None: not a date); dates from 1583 on
    (the proleptic Gregorian calendar, where java's hybrid calendar agrees)."""
    if v is None:
        return None
    m = _DATE.fullmatch(_s(v).strip(" "))
    if not m:
        return None
    y = int(m.group(1))
    mo = int(m.group(2)) if m.group(2) is not None and m.group(2) != "" else (0 if m.group(2) == "" else 1)
    d = int(m.group(3)) if m.group(3) is not None and m.group(3) != "" else (0 if m.group(3) == "" else 1)
    try:
        return (_dt.date(y, mo, d) - _dt.date(1970, 1, 1)).days
    except ValueError:
        return None


def _date_str(days):
    return None if days is None else (_dt.date(1970, 1, 1) + _dt.timedelta(days=days)).isoformat()


def connect():
    con = sqlite3.connect(":memory:")
    con.create_function("soundex", 1, _spark_soundex, deterministic=True)
    con.create_function("regexp_replace", 3, _spark_regexp_replace, deterministic=True)
    con.create_function("regexp_extract", 2, _spark_regexp_extract, deterministic=True)
    con.create_function("regexp_extract", 3, _spark_regexp_extract, deterministic=True)
    con.create_function("to_date", 1, lambda v: _date_str(_days(v)), deterministic=True)
    con.create_function("date_add", 2, lambda v, k: None if _days(v) is None else _date_str(_days(v) + int(k)),
                        deterministic=True)
    con.create_function("date_sub", 2, lambda v, k: None if _days(v) is None else _date_str(_days(v) - int(k)),
                        deterministic=True)
    con.create_function("datediff", 2, lambda a, b: None if _days(a) is None or _days(b) is None else _days(a) - _days(b),
                        deterministic=True)
    con.create_function("jaro_winkler_sim", 2, jaro_winkler, deterministic=True)
    con.create_function("levenshtein", 2, _lev, deterministic=True)
    con.create_function("length", 1, _length, deterministic=True)
    for name, fn in (("lower", _spark_lower), ("lcase", _spark_lower), ("upper", _spark_upper),
                     ("ucase", _spark_upper), ("trim", _spark_trim),
                     ("ltrim", lambda v: _spark_trim(v, "left")), ("rtrim", lambda v: _spark_trim(v, "right"))):
        con.create_function(name, 1, fn, deterministic=True)
    con.create_function("concat", -1, _spark_concat, deterministic=True)
    con.create_function("concat_ws", -1, _spark_concat_ws, deterministic=True)
    for t, fn in _CASTS.items():
        con.create_function(f"spark_cast_{t}", 1, fn, deterministic=True)
    return con


def block(settings, df=None, df_l=None, df_r=None):
    """Candidate pairs as (row_l, row_r) indices into the (possibly concatenated) tables.

    Restates blocking.py:95-160 / 219-268: one inner join per rule, each excluding pairs an
    earlier rule already produced (`AND NOT (ifnull((rule_j), false) ...)`), plus the link-type
    predicate.  Returns (pairs DataFrame, left table, right table)."""
    con = connect()
    lt = settings["link_type"]
    uid = settings.get("unique_id_column_name", "unique_id")
    if lt == "dedupe_only":
        left = right = df.reset_index(drop=True)
    elif lt == "link_only":
        left, right = df_l.reset_index(drop=True), df_r.reset_index(drop=True)
    else:
        left = pd.concat([df_l.assign(_source_table="left"), df_r.assign(_source_table="right")],
                         ignore_index=True)
        right = left
    left.assign(_row=np.arange(len(left))).to_sql("tl", con, index=False)
    right.assign(_row=np.arange(len(right))).to_sql("tr", con, index=False)
    if lt == "dedupe_only":
        where = f"where l.{uid} < r.{uid}"
    elif lt == "link_only":
        where = ""
    else:
        where = (f"where (l._source_table < r._source_table) or "
                 f"(l.{uid} < r.{uid} and l._source_table = r._source_table)")
    rules = settings.get("blocking_rules") or []
    parts = []
    if not rules:
        parts.append(f"select l._row as row_l, r._row as row_r from tl l cross join tr r {where}")
    for k, rule in enumerate(rules):
        prev = " or ".join(f"ifnull(({p}), 0)" for p in rules[:k])
        notprev = f"and not ({prev})" if prev else ""
        parts.append(f"select l._row as row_l, r._row as row_r from tl l inner join tr r on {rule} {notprev} {where}")
    pairs = pd.read_sql(" union all ".join(parts), con)
    return pairs, left, right


def comparison_frame(pairs, left, right):
    l = left.iloc[pairs["row_l"].to_numpy()].reset_index(drop=True).add_suffix("_l")
    r = right.iloc[pairs["row_r"].to_numpy()].reset_index(drop=True).add_suffix("_r")
    return pd.concat([l, r], axis=1)


def sql_gammas(cmp_df, case_expressions):
    """Evaluate each CASE expression over the comparison frame with sqlite (gammas.py:65-89)."""
    con = connect()
    cmp_df = cmp_df.copy()
    for c in cmp_df.columns:
        if cmp_df[c].dtype == object:
            cmp_df[c] = cmp_df[c].where(cmp_df[c].notna(), None)
    cmp_df.to_sql("cmp", con, index=False)
    out = np.empty((len(cmp_df), len(case_expressions)), dtype=np.int8)
    for k, expr in enumerate(case_expressions):
        e = rewrite_casts(spark_literals(_strip_alias(expr)))
        vals = [r[0] for r in con.execute(f"select {e} from cmp").fetchall()]
        out[:, k] = np.array([-99 if v is None else v for v in vals], dtype=np.int64)
    return out


def _strip_alias(expr):
    s = " ".join(expr.split())
    low = s.lower()
    i = low.rfind(" end")
    return s[: i + 4] if i >= 0 else s


def _bayes(ps):
    """term_frequencies.py:21-46: Πp / (Πp + Π(1-p)), products left-associative; x/0 -> NULL."""
    a = ps[0]
    for p in ps[1:]:
        a = a * p
    b = 1.0 - ps[0]
    for p in ps[1:]:
        b = b * (1.0 - p)
    d = a + b
    return float("nan") if d == 0 else a / d


def tf_adjust(cols_l, cols_r, mp, lam):
    """make_adjustment_for_term_frequencies (term_frequencies.py:122-168).

    cols_l / cols_r: list (one per tf column) of per-pair values; mp: per-pair match probability
    (NaN = NULL).  Returns (tf_adjusted_match_prob, [per-column *_adj])."""
    one_minus = float(repr(1 - lam))
    adjs = []
    for vl, vr in zip(cols_l, cols_r):
        acc = {}
        for a, b, p in zip(vl, vr, mp):
            if a is None or b is None or a != b:
                continue
            s = acc.setdefault(a, [0.0, 0])
            if not np.isnan(p):
                s[0] += p
                s[1] += 1
        lookup = {}
        for v, (s, n) in acc.items():
            lookup[v] = float("nan") if n == 0 else _bayes([s / n, one_minus])
        col = []
        for a, b in zip(vl, vr):
            x = lookup.get(a) if (a is not None and b is not None and a == b) else None
            col.append(0.5 if x is None or np.isnan(x) else x)
        adjs.append(np.array(col, dtype=np.float64))
    out = np.array([float("nan") if np.isnan(p) else _bayes([p] + [c[i] for c in adjs])
                    for i, p in enumerate(mp)], dtype=np.float64)
    return out, adjs


def tf_adjust_codes(codes_l, codes_r, mp, lam):
    """tf_adjust for ONE tf column over integer value codes (-1 = NULL), vectorised for pair counts the
    scalar loop cannot take (term_frequencies.py:49-117, the same steps as tf_adjust): per value v,
    adj_lambda = mean mp over pairs with code_l = code_r = v (NULL mp out of sum and count), adj =
    bayes(adj_lambda, 1 - λ), 0.5 where the pair has no lookup (or a NULL one), then
    bayes(mp, adj).  Σmp per value is np.bincount's running sum in pair order, as the scalar loop."""
    codes_l = np.asarray(codes_l, dtype=np.int64)
    codes_r = np.asarray(codes_r, dtype=np.int64)
    n_v = int(max(codes_l.max(initial=-1), codes_r.max(initial=-1))) + 1
    s, c = tf_value_sums(codes_l, codes_r, mp, n_v)
    return tf_adjust_with_sums(codes_l, codes_r, mp, lam, s, c)


def tf_value_sums(codes_l, codes_r, mp, n_values, sums=None, counts=None):
    """Per value v: Σ mp and the count over pairs with code_l = code_r = v and a non-NULL mp
    (term_frequencies.py:49-65).  Added to `sums` / `counts` when given, so the pairs of a large job can be
    taken chunk by chunk."""
    codes_l = np.asarray(codes_l, dtype=np.int64)
    codes_r = np.asarray(codes_r, dtype=np.int64)
    mp = np.asarray(mp, dtype=np.float64)
    good = (codes_l >= 0) & (codes_l == codes_r) & ~np.isnan(mp)
    s = np.bincount(codes_l[good], weights=mp[good], minlength=n_values)
    c = np.bincount(codes_l[good], minlength=n_values)
    if sums is None:
        return s, c
    sums += s
    counts += c
    return sums, counts


def tf_adjust_with_sums(codes_l, codes_r, mp, lam, s, c):
    """tf_adjust_codes' adjustment of the pairs given, from per-value sums and counts over all the job's
    pairs (tf_value_sums; term_frequencies.py:68-117)."""
    codes_l = np.asarray(codes_l, dtype=np.int64)
    codes_r = np.asarray(codes_r, dtype=np.int64)
    mp = np.asarray(mp, dtype=np.float64)
    one_minus = float(repr(1 - lam))
    ok = (codes_l >= 0) & (codes_l == codes_r)
    n_v = len(s)
    with np.errstate(invalid="ignore", divide="ignore"):
        adj_lambda = np.where(c > 0, s / np.maximum(c, 1), np.nan)
        tnum = adj_lambda * one_minus
        tden = tnum + (1.0 - adj_lambda) * (1.0 - one_minus)
        tab = np.where(tden == 0, np.nan, tnum / tden)
        adj = np.full(len(mp), 0.5)
        look = tab[np.where(ok, codes_l, 0)] if n_v else np.full(len(mp), np.nan)
        sel = ok & ~np.isnan(look)
        adj[sel] = look[sel]
        num = mp * adj
        den = num + (1.0 - mp) * (1.0 - adj)
        out = np.where(den == 0, np.nan, num / den)
    out[np.isnan(mp)] = np.nan
    return out, adj
