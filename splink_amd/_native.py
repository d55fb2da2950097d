"""ctypes binding to libsplink_hip.so (the C ABI declared in include/splink_hip.h).

There is no CPU fallback: if the library or a gfx950 device is missing, every product
entry point raises `NativeUnavailable`.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPLINK_AMD_LIB", os.path.join(_HERE, "libsplink_hip.so"))

SPK_OK = 0
SPK_E_INVALID = -1
SPK_E_HIP = -2
SPK_E_OOM = -3
SPK_E_STATE = -4
SPK_E_LIMIT = -5

LINK_TYPES = {"dedupe_only": 0, "link_only": 1, "link_and_dedupe": 2}

# ---- C structs mirrored as numpy structured dtypes (same layout as splink_hip.h) ----------
OPERAND_DTYPE = np.dtype([("kind", "<i4"), ("side", "<i4"), ("col", "<i4"), ("lit", "<i4"), ("num", "<f8"),
                          ("has_num_default", "<i4"), ("substr_start", "<i4"), ("substr_len", "<i4"),
                          ("pad", "<i4")], align=True)
INSTR_DTYPE = np.dtype([("op", "<i4"), ("a", "<i4"), ("b", "<i4"), ("cmp", "<i4"), ("i0", "<i4"), ("pad", "<i4"),
                        ("t", "<f8")], align=True)
PROGRAM_DTYPE = np.dtype([("n_levels", "<i4"), ("else_level", "<i4"), ("n_when", "<i4"), ("first_when", "<i4")],
                         align=True)
KEY_TERM_DTYPE = np.dtype([("raw_l", "<i4"), ("raw_r", "<i4"), ("l_substr_start", "<i4"), ("l_substr_len", "<i4"),
                           ("r_substr_start", "<i4"), ("r_substr_len", "<i4")], align=True)
assert KEY_TERM_DTYPE.itemsize == 24
assert OPERAND_DTYPE.itemsize == 40 and INSTR_DTYPE.itemsize == 32 and PROGRAM_DTYPE.itemsize == 16

OP = {"ISNULL": 1, "NOTNULL": 2, "STR_CMP": 3, "NUM_CMP": 4, "JW": 5, "LEV": 6, "LEVRATIO": 7, "ABSDIFF": 8,
      "PERCDIFF": 9, "CONST": 10, "LEN": 11, "AND": 20, "OR": 21, "NOT": 22}
CMP = {"=": 0, "==": 0, "!=": 1, "<>": 1, "<": 2, "<=": 3, ">": 4, ">=": 5}

EXPORTS = [
    "spk_last_error", "spk_version", "spk_device_count", "spk_ctx_create", "spk_ctx_destroy", "spk_ctx_set_stream",
    "spk_ctx_sync", "spk_ctx_set_link_type", "spk_ctx_kernel_ms", "spk_ctx_enable_timing", "spk_table_create",
    "spk_table_add_utf8", "spk_table_add_float64", "spk_table_set_rank", "spk_table_set_key", "spk_block",
    "spk_pairs_count", "spk_pairs_copy", "spk_pairs_load", "spk_gammas", "spk_gammas_copy", "spk_gammas_load",
    "spk_n_patterns", "spk_gammas_deferred", "spk_em_histogram", "spk_em_finalize", "spk_em_iteration", "spk_score",
    "spk_tf_accumulate", "spk_tf_apply", "spk_jaro_winkler_sim", "spk_levenshtein", "spk_gammas_exact_counts",
    "spk_gammas_set_simple", "spk_gammas_exact_list", "spk_gammas_simple_count", "spk_em_set_lane_histogram", "spk_table_set_rank_null",
    "spk_gammas_view_regions", "spk_ctx_lds_per_block", "spk_ctx_memory", "spk_raw_utf8", "spk_raw_i64", "spk_key_build", "spk_rank_from_raw", "spk_cluster", "spk_table_add_raw_utf8",
    "spk_gammas_implied_pairs", "spk_tf_column_values", "spk_tf_accumulate_column", "spk_tf_apply_columns", "spk_tf_copy", "spk_tf_set_mode",
    "spk_tf_accumulate_exact", "spk_tf_accumulate_column_exact", "spk_tf_limbs_to_sum", "spk_tf_scales",
    "spk_tf_scales_column", "spk_raw_utf8_arrow", "spk_raw_utf8_arrow_chunks", "spk_table_digest", "spk_raw_release",
    "spk_em_iteration_start", "spk_em_iteration_wait", "spk_ctx_kernel_ms_done", "spk_em_histogram_async",
    "spk_em_finalize_start", "spk_gammas_exact_ms", "spk_gammas_set_window", "spk_gammas_windows", "spk_gammas_set_streams", "spk_gammas_set_graph",
    "spk_gammas_graph_launches",
    "spk_gammas_set_lev_kernel",
]
TF_LIMBS = 14  # SPK_TF_LIMBS


class NativeUnavailable(RuntimeError):
    """libsplink_hip.so or a gfx950 HIP device is unavailable (there is no CPU fallback)."""


_lib = None


def load_library():
    """Load libsplink_hip.so (no device needed)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    lib.spk_last_error.restype = ctypes.c_char_p
    lib.spk_ctx_destroy.restype = None
    for name in EXPORTS:
        getattr(lib, name)  # raises AttributeError when a declared symbol is missing
    _lib = lib
    return lib


def tf_limbs_to_sum(limbs, scale) -> np.ndarray:
    """Σmp per value from fixed-point accumulators and the values' scales (host only, no device)."""
    lib = load_library()
    limbs = np.ascontiguousarray(limbs, dtype=np.int64).reshape(-1, TF_LIMBS)
    scale = np.ascontiguousarray(scale, dtype=np.int32)
    assert len(scale) == len(limbs)
    out = np.zeros(max(len(limbs), 1), dtype=np.float64)
    check(lib.spk_tf_limbs_to_sum(ctypes.c_int64(len(limbs)), _ptr(limbs), _ptr(scale), _ptr(out)),
          "spk_tf_limbs_to_sum")
    return out[:len(limbs)]


TF_NO_SCALE = np.iinfo(np.int32).min  # a value without a positive term


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int(0)
    lib.spk_device_count(ctypes.byref(n))
    return n.value


def _ptr(a):
    return ctypes.c_void_p(0) if a is None else ctypes.c_void_p(a.ctypes.data)


def check(rc: int, what: str):
    if rc == SPK_OK:
        return
    msg = load_library().spk_last_error().decode("utf-8", "replace")
    if rc in (SPK_E_INVALID, SPK_E_LIMIT):
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what} failed ({rc}): {msg}")


class Context:
    """One spk_ctx: one device, one stream, one set of tables / pairs / codes."""

    def __init__(self, device: int = 0):
        lib = load_library()
        if device_count() <= device:
            raise NativeUnavailable(f"no HIP device {device} visible (splink_amd needs an MI355X / gfx950)")
        h = ctypes.c_void_p()
        check(lib.spk_ctx_create(ctypes.c_int(device), ctypes.byref(h)), "spk_ctx_create")
        self._h = h
        self._lib = lib
        self.device = device

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.spk_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- calls ------------------------------------------------------------------------
    def set_stream(self, stream_ptr: int):
        check(self._lib.spk_ctx_set_stream(self._h, ctypes.c_void_p(stream_ptr)), "spk_ctx_set_stream")

    def sync(self):
        check(self._lib.spk_ctx_sync(self._h), "spk_ctx_sync")

    def set_link_type(self, link_type: int):
        check(self._lib.spk_ctx_set_link_type(self._h, ctypes.c_int(link_type)), "spk_ctx_set_link_type")

    def enable_timing(self, on: bool = True, exact: bool = False):
        """HIP-event timing of the kernel families; exact=True also times each column's exact-pass launch."""
        check(self._lib.spk_ctx_enable_timing(self._h, ctypes.c_int((2 if exact else 1) if on else 0)),
              "spk_ctx_enable_timing")

    def kernel_ms(self):
        out = np.zeros(5, dtype=np.float64)
        check(self._lib.spk_ctx_kernel_ms(self._h, _ptr(out)), "spk_ctx_kernel_ms")
        return dict(zip(["block", "gamma", "em_hist", "em_final", "score"], out.tolist()))

    def kernel_ms_done(self):
        """kernel_ms without synchronising: per family the newest launch that has completed (-1 = none)."""
        out = np.zeros(5, dtype=np.float64)
        check(self._lib.spk_ctx_kernel_ms_done(self._h, _ptr(out)), "spk_ctx_kernel_ms_done")
        return dict(zip(["block", "gamma", "em_hist", "em_final", "score"], out.tolist()))

    def table_create(self, side: int, n_rows: int, n_cols: int):
        check(self._lib.spk_table_create(self._h, ctypes.c_int(side), ctypes.c_int64(n_rows), ctypes.c_int(n_cols)),
              "spk_table_create")

    def table_add_utf8(self, side, col, offsets, data, valid, value_ids=None):
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, dtype=np.uint8)
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
        ids = None if value_ids is None else np.ascontiguousarray(value_ids, dtype=np.int64)
        check(self._lib.spk_table_add_utf8(self._h, ctypes.c_int(side), ctypes.c_int(col), _ptr(offsets), _ptr(data),
                                           _ptr(valid), _ptr(ids)), "spk_table_add_utf8")

    def table_add_float64(self, side, col, values, valid):
        values = np.ascontiguousarray(values, dtype=np.float64)
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
        check(self._lib.spk_table_add_float64(self._h, ctypes.c_int(side), ctypes.c_int(col), _ptr(values),
                                              _ptr(valid)), "spk_table_add_float64")

    def table_set_rank(self, side, rank):
        rank = np.ascontiguousarray(rank, dtype=np.int64)
        check(self._lib.spk_table_set_rank(self._h, ctypes.c_int(side), _ptr(rank)), "spk_table_set_rank")

    def table_set_rank_null(self, side, divisor):
        check(self._lib.spk_table_set_rank_null(self._h, ctypes.c_int(side), ctypes.c_int64(divisor)),
              "spk_table_set_rank_null")

    # ---- device ingest ---------------------------------------------------------------------
    def raw_utf8(self, raw, offsets, data, valid):
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if data.size == 0:
            data = np.zeros(1, dtype=np.uint8)
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
        check(self._lib.spk_raw_utf8(self._h, ctypes.c_int(raw), ctypes.c_int64(len(offsets) - 1), _ptr(offsets),
                                     _ptr(data), _ptr(valid)), "spk_raw_utf8")

    def raw_utf8_arrow(self, raw, n, offsets, data, bitmap=None, bit_offset=0):
        """Arrow buffers as numpy views (no copies): offsets int64[n+1] (any base), data uint8, validity bitmap
        (None = no NULLs; bit_offset -1 = one byte per row)."""
        check(self._lib.spk_raw_utf8_arrow(self._h, ctypes.c_int(raw), ctypes.c_int64(n), _ptr(offsets), _ptr(data),
                                           _ptr(bitmap), ctypes.c_int64(bit_offset), ctypes.c_int(0)),
              "spk_raw_utf8_arrow")

    def raw_utf8_arrow_chunks(self, raw, views, rows):
        """A chunked Arrow column: views[c] = arrow_views(chunk c) (offsets, data, bitmap or None, bit offset),
        rows[c] its row count; the chunks' rows are concatenated on the device."""
        nc = len(views)
        c_rows = (ctypes.c_int64 * nc)(*[int(r) for r in rows])
        c_off = (ctypes.c_void_p * nc)(*[_ptr(v[0]).value for v in views])
        c_data = (ctypes.c_void_p * nc)(*[_ptr(v[1]).value for v in views])
        c_valid = (ctypes.c_void_p * nc)(*[_ptr(v[2]).value if v[2] is not None else None for v in views])
        c_bit = (ctypes.c_int64 * nc)(*[int(v[3]) if v[2] is not None else 0 for v in views])
        check(self._lib.spk_raw_utf8_arrow_chunks(self._h, ctypes.c_int(raw), ctypes.c_int(nc), c_rows, c_off, c_data,
                                                  c_valid, c_bit), "spk_raw_utf8_arrow_chunks")

    def raw_utf8_device(self, raw, n, d_offsets, d_data, d_valid_bytes):
        """The same from device buffers (int pointers: offsets int64[n+1], data, one validity byte per row)."""
        check(self._lib.spk_raw_utf8_arrow(self._h, ctypes.c_int(raw), ctypes.c_int64(n), ctypes.c_void_p(d_offsets),
                                           ctypes.c_void_p(d_data), ctypes.c_void_p(d_valid_bytes),
                                           ctypes.c_int64(-1), ctypes.c_int(1)), "spk_raw_utf8_arrow")

    def raw_release(self, raw: int):
        check(self._lib.spk_raw_release(self._h, ctypes.c_int(raw)), "spk_raw_release")

    def table_digest(self, side: int) -> int:
        out = ctypes.c_uint64(0)
        check(self._lib.spk_table_digest(self._h, ctypes.c_int(side), ctypes.byref(out)), "spk_table_digest")
        return out.value

    def raw_i64(self, raw, values, valid):
        values = np.ascontiguousarray(values, dtype=np.int64)
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
        if values.size == 0:
            values, valid = np.zeros(1, np.int64), np.zeros(1, np.uint8)
            n = 0
        else:
            n = len(values)
        check(self._lib.spk_raw_i64(self._h, ctypes.c_int(raw), ctypes.c_int64(n), _ptr(values), _ptr(valid)),
              "spk_raw_i64")

    def key_build(self, rule, terms):
        t = np.array([tuple(x) for x in terms], dtype=KEY_TERM_DTYPE)
        check(self._lib.spk_key_build(self._h, ctypes.c_int(rule), ctypes.c_int(len(t)), _ptr(t)), "spk_key_build")

    def rank_from_raw(self, raw_uid, right_from=-1):
        check(self._lib.spk_rank_from_raw(self._h, ctypes.c_int(raw_uid), ctypes.c_int64(right_from)),
              "spk_rank_from_raw")

    def cluster(self, n0, n1=None):
        p0 = np.empty(max(n0, 1), dtype=np.int32)
        p1 = np.empty(max(n1 or 0, 1), dtype=np.int32) if n1 is not None else None
        check(self._lib.spk_cluster(self._h, _ptr(p0), _ptr(p1)), "spk_cluster")
        return p0[:n0], (p1[:n1] if p1 is not None else None)

    def table_add_raw_utf8(self, col, raw0, raw1=-1):
        check(self._lib.spk_table_add_raw_utf8(self._h, ctypes.c_int(col), ctypes.c_int(raw0), ctypes.c_int(raw1)),
              "spk_table_add_raw_utf8")

    def table_set_key(self, side, rule, which, keys):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        check(self._lib.spk_table_set_key(self._h, ctypes.c_int(side), ctypes.c_int(rule), ctypes.c_int(which),
                                          _ptr(keys)), "spk_table_set_key")

    def block(self, link_type: int, symmetric, shard: int = 0, n_shards: int = 1):
        sym = np.ascontiguousarray(symmetric, dtype=np.int32)
        n_pairs = ctypes.c_int64(0)
        n_total = ctypes.c_int64(0)
        check(self._lib.spk_block(self._h, ctypes.c_int(link_type), ctypes.c_int(len(sym)), _ptr(sym),
                                  ctypes.c_int(shard), ctypes.c_int(n_shards), ctypes.byref(n_pairs),
                                  ctypes.byref(n_total)), "spk_block")
        return n_pairs.value, n_total.value

    def pairs_count(self) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.spk_pairs_count(self._h, ctypes.byref(n)), "spk_pairs_count")
        return n.value

    def pairs_copy(self, start: int = 0, count: int | None = None):
        if count is None:
            count = self.pairs_count() - start
        l = np.empty(count, dtype=np.int32)
        r = np.empty(count, dtype=np.int32)
        check(self._lib.spk_pairs_copy(self._h, ctypes.c_int64(start), ctypes.c_int64(count), _ptr(l), _ptr(r)),
              "spk_pairs_copy")
        return l, r

    def pairs_load(self, rows_l, rows_r):
        rows_l = np.ascontiguousarray(rows_l, dtype=np.int32)
        rows_r = np.ascontiguousarray(rows_r, dtype=np.int32)
        check(self._lib.spk_pairs_load(self._h, ctypes.c_int64(len(rows_l)), _ptr(rows_l), _ptr(rows_r)),
              "spk_pairs_load")

    @staticmethod
    def gammas_args(programs, when_first, when_n, when_level, instrs, operands, lit_offsets, lit_bytes):
        """The spk_gammas argument list, converted once (cached by the caller across calls)."""
        programs = np.ascontiguousarray(programs, dtype=PROGRAM_DTYPE)
        wf = np.ascontiguousarray(when_first, dtype=np.int32)
        wn = np.ascontiguousarray(when_n, dtype=np.int32)
        wl = np.ascontiguousarray(when_level, dtype=np.int32)
        instrs = np.ascontiguousarray(instrs, dtype=INSTR_DTYPE)
        operands = np.ascontiguousarray(operands, dtype=OPERAND_DTYPE)
        lo = np.ascontiguousarray(lit_offsets, dtype=np.int64)
        lb = np.ascontiguousarray(lit_bytes, dtype=np.uint8)
        if lb.size == 0:
            lb = np.zeros(1, dtype=np.uint8)
        keep = (programs, wf, wn, wl, instrs, operands, lo, lb)
        c_args = (ctypes.c_int(len(programs)), _ptr(programs), ctypes.c_int(len(wf)), _ptr(wf), _ptr(wn), _ptr(wl),
                  ctypes.c_int(len(instrs)), _ptr(instrs), ctypes.c_int(len(operands)), _ptr(operands),
                  ctypes.c_int(len(lo) - 1), _ptr(lo), _ptr(lb))
        return keep, c_args

    def gammas_native(self, args):
        check(self._lib.spk_gammas(self._h, *args[1]), "spk_gammas")

    def gammas(self, programs, when_first, when_n, when_level, instrs, operands, lit_offsets, lit_bytes):
        programs = np.ascontiguousarray(programs, dtype=PROGRAM_DTYPE)
        wf = np.ascontiguousarray(when_first, dtype=np.int32)
        wn = np.ascontiguousarray(when_n, dtype=np.int32)
        wl = np.ascontiguousarray(when_level, dtype=np.int32)
        instrs = np.ascontiguousarray(instrs, dtype=INSTR_DTYPE)
        operands = np.ascontiguousarray(operands, dtype=OPERAND_DTYPE)
        lo = np.ascontiguousarray(lit_offsets, dtype=np.int64)
        lb = np.ascontiguousarray(lit_bytes, dtype=np.uint8)
        if lb.size == 0:
            lb = np.zeros(1, dtype=np.uint8)
        check(self._lib.spk_gammas(self._h, ctypes.c_int(len(programs)), _ptr(programs), ctypes.c_int(len(wf)),
                                   _ptr(wf), _ptr(wn), _ptr(wl), ctypes.c_int(len(instrs)), _ptr(instrs),
                                   ctypes.c_int(len(operands)), _ptr(operands), ctypes.c_int(len(lo) - 1), _ptr(lo),
                                   _ptr(lb)), "spk_gammas")

    def gammas_load(self, n_levels, gammas):
        nl = np.ascontiguousarray(n_levels, dtype=np.int32)
        g = np.ascontiguousarray(gammas, dtype=np.int8)
        check(self._lib.spk_gammas_load(self._h, ctypes.c_int(len(nl)), _ptr(nl), ctypes.c_int64(g.shape[0]), _ptr(g)),
              "spk_gammas_load")

    def gammas_copy(self, K: int, start: int, count: int):
        out = np.empty((count, K), dtype=np.int8)
        check(self._lib.spk_gammas_copy(self._h, ctypes.c_int64(start), ctypes.c_int64(count), _ptr(out)),
              "spk_gammas_copy")
        return out

    def n_patterns(self) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.spk_n_patterns(self._h, ctypes.byref(n)), "spk_n_patterns")
        return n.value

    def gammas_deferred(self) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.spk_gammas_deferred(self._h, ctypes.byref(n)), "spk_gammas_deferred")
        return n.value

    def gammas_exact_counts(self, K: int):
        out = np.zeros(max(K, 1), dtype=np.int64)
        check(self._lib.spk_gammas_exact_counts(self._h, _ptr(out), ctypes.c_int(len(out))), "spk_gammas_exact_counts")
        return out[:K].tolist()

    def gammas_exact_list(self, k: int, n: int):
        out = np.empty(int(n), dtype=np.int32)
        check(self._lib.spk_gammas_exact_list(self._h, ctypes.c_int(k), _ptr(out), ctypes.c_int64(int(n))),
              "spk_gammas_exact_list")
        return out

    def gammas_implied_pairs(self, K: int):
        out = np.zeros(max(K, 1), dtype=np.int64)
        check(self._lib.spk_gammas_implied_pairs(self._h, _ptr(out), ctypes.c_int(len(out))), "spk_gammas_implied_pairs")
        return out[:K].tolist()

    def gammas_set_simple(self, mode):
        """1 / True: template-shaped columns through the filter kernel, 0: every column through the interpreter;
        + 10: rule 1's pairs never read the view-ordered image, + 20: always (tests)."""
        check(self._lib.spk_gammas_set_simple(self._h, ctypes.c_int(int(mode))), "spk_gammas_set_simple")

    def gammas_set_window(self, pairs: int):
        """Cap spk_gammas' ordinal windows at `pairs` (0 = default, just under 2^31; for testing)."""
        check(self._lib.spk_gammas_set_window(self._h, ctypes.c_int64(int(pairs))), "spk_gammas_set_window")

    def gammas_set_streams(self, streams: int, min_pairs: int = 1 << 22):
        """spk_gammas' two-stream split: 2 streams (default) for pair sets of at least min_pairs, or 1."""
        check(self._lib.spk_gammas_set_streams(self._h, ctypes.c_int(int(streams)), ctypes.c_int64(int(min_pairs))),
              "spk_gammas_set_streams")

    def gammas_set_graph(self, on: bool):
        """Replay unchanged comparison passes from a captured HIP graph (default off: slower than direct launches)."""
        check(self._lib.spk_gammas_set_graph(self._h, ctypes.c_int(1 if on else 0)), "spk_gammas_set_graph")

    def gammas_graph_launches(self) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.spk_gammas_graph_launches(self._h, ctypes.byref(n)), "spk_gammas_graph_launches")
        return n.value

    def gammas_windows(self) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.spk_gammas_windows(self._h, ctypes.byref(n)), "spk_gammas_windows")
        return n.value

    def gammas_set_lev_kernel(self, mode: int):
        """Levenshtein exact pass (same codes; A/B tests): 2 lane refill in free-text columns, one cell per lane
        elsewhere (default); 1 lane refill everywhere; 0 one cell per lane everywhere; 3 as 2 without the
        character-bag decisions before the refill pass."""
        check(self._lib.spk_gammas_set_lev_kernel(self._h, ctypes.c_int(int(mode))), "spk_gammas_set_lev_kernel")

    def lds_per_block(self) -> int:
        n = ctypes.c_int(0)
        check(self._lib.spk_ctx_lds_per_block(self._h, ctypes.byref(n)), "spk_ctx_lds_per_block")
        return n.value

    MEMORY_PARTS = ("raw_columns", "record_encodings", "row_images", "pairs", "codes", "work_lists", "em_score_tf",
                    "total")

    def memory(self) -> dict:
        """Device bytes the context holds, by what they store (spk_ctx_memory)."""
        out = np.zeros(8, dtype=np.int64)
        check(self._lib.spk_ctx_memory(self._h, _ptr(out)), "spk_ctx_memory")
        return dict(zip(self.MEMORY_PARTS, [int(x) for x in out]))

    def gammas_view_regions(self) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.spk_gammas_view_regions(self._h, ctypes.byref(n)), "spk_gammas_view_regions")
        return n.value

    def gammas_exact_ms(self, n: int):
        out = np.zeros(max(n, 1), dtype=np.float64)
        check(self._lib.spk_gammas_exact_ms(self._h, _ptr(out), ctypes.c_int(n)), "spk_gammas_exact_ms")
        return out[:n].tolist()

    def gammas_simple_count(self) -> int:
        n = ctypes.c_int(0)
        check(self._lib.spk_gammas_simple_count(self._h, ctypes.byref(n)), "spk_gammas_simple_count")
        return n.value

    def em_set_lane_histogram(self, on):
        """True / 1: lane-private counters, release fence before each last-arriver ticket (default); False / 0:
        wave-ballot histogram; 2: lane counters without the fence (A/B)."""
        check(self._lib.spk_em_set_lane_histogram(self._h, ctypes.c_int(int(on))), "spk_em_set_lane_histogram")

    def em_histogram(self, d_hist_ptr: int = 0):
        check(self._lib.spk_em_histogram(self._h, ctypes.c_void_p(d_hist_ptr)), "spk_em_histogram")

    def em_histogram_async(self, d_hist_ptr: int):
        check(self._lib.spk_em_histogram_async(self._h, ctypes.c_void_p(d_hist_ptr)), "spk_em_histogram_async")

    def em_finalize_start(self, d_hist_ptr, lam, one_minus, m, u, n_stats):
        m = np.ascontiguousarray(m, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        check(self._lib.spk_em_finalize_start(self._h, ctypes.c_void_p(d_hist_ptr), ctypes.c_double(lam),
                                              ctypes.c_double(one_minus), _ptr(m), _ptr(u), ctypes.c_int(n_stats)),
              "spk_em_finalize_start")

    def em_finalize(self, d_hist_ptr, lam, one_minus, m, u, n_stats):
        m = np.ascontiguousarray(m, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.zeros(n_stats, dtype=np.float64)
        check(self._lib.spk_em_finalize(self._h, ctypes.c_void_p(d_hist_ptr), ctypes.c_double(lam),
                                        ctypes.c_double(one_minus), _ptr(m), _ptr(u), _ptr(out),
                                        ctypes.c_int(n_stats)), "spk_em_finalize")
        return out

    def em_iteration(self, lam, one_minus, m, u, n_stats):
        """One E+M iteration on this GPU's pairs in one launch (histogram, E-step per pattern, M-step sums)."""
        m = np.ascontiguousarray(m, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = self._stats_buf(n_stats)
        check(self._lib.spk_em_iteration(self._h, ctypes.c_double(lam), ctypes.c_double(one_minus), _ptr(m), _ptr(u),
                                         _ptr(out), ctypes.c_int(n_stats)), "spk_em_iteration")
        return out

    def em_iteration_start(self, lam, one_minus, m, u, n_stats):
        """Enqueue one E+M iteration (spk_em_iteration_start); em_iteration_wait returns its statistics."""
        m = np.ascontiguousarray(m, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        check(self._lib.spk_em_iteration_start(self._h, ctypes.c_double(lam), ctypes.c_double(one_minus), _ptr(m),
                                               _ptr(u), ctypes.c_int(n_stats)), "spk_em_iteration_start")

    def em_iteration_wait(self, n_stats):
        out = self._stats_buf(n_stats)
        check(self._lib.spk_em_iteration_wait(self._h, _ptr(out), ctypes.c_int(n_stats)), "spk_em_iteration_wait")
        return out

    def _stats_buf(self, n_stats):
        return np.zeros(n_stats, dtype=np.float64)

    def score(self, lam, one_minus, m, u, start=0, count=0, want_host=True):
        m = np.ascontiguousarray(m, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.empty(count, dtype=np.float64) if want_host else None
        check(self._lib.spk_score(self._h, ctypes.c_double(lam), ctypes.c_double(one_minus), _ptr(m), _ptr(u),
                                  ctypes.c_int64(start), ctypes.c_int64(count), _ptr(out)), "spk_score")
        return out

    def _udf(self, fn, left, right):
        from .table import encode_utf8
        import pandas as pd
        lo, ld, _ = encode_utf8(pd.Series(list(left), dtype=object))
        ro, rd, _ = encode_utf8(pd.Series(list(right), dtype=object))
        ld = ld if ld.size else np.zeros(1, np.uint8)
        rd = rd if rd.size else np.zeros(1, np.uint8)
        out = np.empty(len(lo) - 1, dtype=np.float64)
        check(getattr(self._lib, fn)(self._h, ctypes.c_int64(len(out)), _ptr(lo), _ptr(ld), _ptr(ro), _ptr(rd),
                                     _ptr(out)), fn)
        return out

    def jaro_winkler_sim(self, left, right):
        return self._udf("spk_jaro_winkler_sim", left, right)

    def levenshtein(self, left, right):
        return self._udf("spk_levenshtein", left, right)

    def tf_accumulate(self, n_values, ids0, ids1):
        ids0 = np.ascontiguousarray(ids0, dtype=np.int64)
        ids1 = np.ascontiguousarray(ids1, dtype=np.int64)
        s = np.zeros(max(n_values, 1), dtype=np.float64)
        c = np.zeros(max(n_values, 1), dtype=np.int64)
        check(self._lib.spk_tf_accumulate(self._h, ctypes.c_int64(n_values), _ptr(ids0), _ptr(ids1), _ptr(s), _ptr(c)),
              "spk_tf_accumulate")
        return s[:n_values], c[:n_values]

    def tf_scales(self, n_values, ids0, ids1):
        """Per-value scales (int32: ilogb of the value's largest mp + 1) of this context's pairs; ranks
        holding shards of the pairs all-reduce them with MAX before tf_accumulate_exact."""
        ids0 = np.ascontiguousarray(ids0, dtype=np.int64)
        ids1 = np.ascontiguousarray(ids1, dtype=np.int64)
        sc = np.zeros(max(n_values, 1), dtype=np.int32)
        check(self._lib.spk_tf_scales(self._h, ctypes.c_int64(n_values), _ptr(ids0), _ptr(ids1), _ptr(sc)),
              "spk_tf_scales")
        return sc[:n_values]

    def tf_scales_column(self, col: int, n_values: int):
        sc = np.zeros(max(n_values, 1), dtype=np.int32)
        check(self._lib.spk_tf_scales_column(self._h, ctypes.c_int(col), ctypes.c_int64(n_values), _ptr(sc)),
              "spk_tf_scales_column")
        return sc[:n_values]

    def tf_accumulate_exact(self, n_values, ids0, ids1, scale):
        """Fixed-point per-value Σmp accumulators (int64 [n_values, TF_LIMBS]) relative to 2^scale, and counts:
        exact, so ranks holding shards of the pairs sum them (all-reduce) before tf_limbs_to_sum."""
        ids0 = np.ascontiguousarray(ids0, dtype=np.int64)
        ids1 = np.ascontiguousarray(ids1, dtype=np.int64)
        scale = np.ascontiguousarray(scale, dtype=np.int32)
        limbs = np.zeros((max(n_values, 1), TF_LIMBS), dtype=np.int64)
        c = np.zeros(max(n_values, 1), dtype=np.int64)
        check(self._lib.spk_tf_accumulate_exact(self._h, ctypes.c_int64(n_values), _ptr(ids0), _ptr(ids1), _ptr(scale),
                                                _ptr(limbs), _ptr(c)), "spk_tf_accumulate_exact")
        return limbs[:n_values], c[:n_values]

    def tf_accumulate_column_exact(self, col: int, n_values: int, scale):
        scale = np.ascontiguousarray(scale, dtype=np.int32)
        limbs = np.zeros((max(n_values, 1), TF_LIMBS), dtype=np.int64)
        c = np.zeros(max(n_values, 1), dtype=np.int64)
        check(self._lib.spk_tf_accumulate_column_exact(self._h, ctypes.c_int(col), ctypes.c_int64(n_values), _ptr(scale),
                                                       _ptr(limbs), _ptr(c)), "spk_tf_accumulate_column_exact")
        return limbs[:n_values], c[:n_values]

    def tf_column_values(self, col: int) -> int:
        n = ctypes.c_int64(0)
        check(self._lib.spk_tf_column_values(self._h, ctypes.c_int(col), ctypes.byref(n)), "spk_tf_column_values")
        return n.value

    def tf_accumulate_column(self, col: int, n_values: int):
        s = np.zeros(max(n_values, 1), dtype=np.float64)
        c = np.zeros(max(n_values, 1), dtype=np.int64)
        check(self._lib.spk_tf_accumulate_column(self._h, ctypes.c_int(col), ctypes.c_int64(n_values), _ptr(s), _ptr(c)),
              "spk_tf_accumulate_column")
        return s[:n_values], c[:n_values]

    def tf_apply_columns(self, cols, tables, start, count, want_adj=True, want_host=True):
        """want_host=False: tf_adjusted_match_prob stays on the device (tf_copy reads ranges of it)."""
        n = len(tables)
        keep = [np.ascontiguousarray(t, dtype=np.float64) if len(t) else np.zeros(1) for t in tables]
        tabs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in keep])
        sizes = np.array([len(t) for t in tables], dtype=np.int64)
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        out = np.empty(count, dtype=np.float64) if want_host else None
        adj = np.empty((count, n), dtype=np.float64) if want_adj else None
        check(self._lib.spk_tf_apply_columns(self._h, ctypes.c_int(n), _ptr(cols), tabs, _ptr(sizes),
                                             ctypes.c_int64(start), ctypes.c_int64(count), _ptr(out), _ptr(adj)),
              "spk_tf_apply_columns")
        return out, adj

    def tf_set_mode(self, mode: int):
        check(self._lib.spk_tf_set_mode(self._h, ctypes.c_int(mode)), "spk_tf_set_mode")

    def tf_copy(self, start, count):
        out = np.empty(count, dtype=np.float64)
        check(self._lib.spk_tf_copy(self._h, ctypes.c_int64(start), ctypes.c_int64(count), _ptr(out)), "spk_tf_copy")
        return out

    def tf_apply(self, ids0_list, ids1_list, tables, start, count, want_adj=True):
        n = len(tables)
        keep = [np.ascontiguousarray(a, dtype=np.int64) for a in ids0_list] + \
               [np.ascontiguousarray(a, dtype=np.int64) for a in ids1_list] + \
               [np.ascontiguousarray(t, dtype=np.float64) if len(t) else np.zeros(1) for t in tables]
        P = ctypes.c_void_p * n
        ids0 = P(*[a.ctypes.data for a in keep[:n]])
        ids1 = P(*[a.ctypes.data for a in keep[n:2 * n]])
        tabs = P(*[a.ctypes.data for a in keep[2 * n:]])
        sizes = np.array([len(t) for t in tables], dtype=np.int64)
        out = np.empty(count, dtype=np.float64)
        adj = np.empty((count, n), dtype=np.float64) if want_adj else None
        check(self._lib.spk_tf_apply(self._h, ctypes.c_int(n), ids0, ids1, tabs, _ptr(sizes), ctypes.c_int64(start),
                                     ctypes.c_int64(count), _ptr(out), _ptr(adj)), "spk_tf_apply")
        return out, adj
