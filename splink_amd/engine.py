"""Device jobs: one spk_ctx per linkage job (record tables, candidate pairs, comparison codes).

This is the executor that replaces Spark's L0 for the hot path:
blocking, comparison vectors, EM and scoring run in libsplink_hip.so on the GPU; Python only
prepares buffers, compiles settings and keeps the reference's model semantics.

Multi-GPU: one process per GPU (torchrun).  When torch.distributed is initialised with more
than one rank, every rank builds the same record tables, generates only its shard of the
candidate-pair ordinal space, and each EM iteration all-reduces the comparison-pattern
histogram (an exact integer sum) with RCCL, so every rank computes identical parameters.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional

import numpy as np
import pandas as pd

from . import _native as N
from . import distributed as D
from . import table as T
from .compiler import CompiledComparisons, Schema, compile_comparisons, compile_rule


N_HEAD = 5  # spk_em_finalize statistics header: [Σmp, rows, non-null rows, Σ ln(..), non-null ln rows]


def default_device() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def session_device(spark) -> int:
    dev = getattr(spark, "device", None)
    return default_device() if dev is None else int(dev)


def distributed_shard():
    """(rank, world_size) when running under torch.distributed with >1 rank, else (0, 1)."""
    return D.shard()


def quantise(p):
    """The E-step renders each m / u as `cast({p:.35f} as double)` (expectation_step.py:212).

    For |p| >= 1e-18 the 35 decimals hold >= 18 significant digits, and any correctly rounded decimal
    of >= 17 significant digits parses back to the same double, so only smaller values (and NaN /
    inf, which fail both tests) go through the text round trip."""
    if p >= 1e-18 or p <= -1e-18 or p == 0:
        return float(p)
    return float(f"{p:.35f}")


def f32(x):
    """`cast(... as float)` of the M-step (maximisation_step.py:19, 68-69)."""
    return None if x is None else float(np.float32(x))


def f32_many(xs):
    """f32 over a list (one numpy conversion instead of one per value); None stays None."""
    idx = [i for i, x in enumerate(xs) if x is not None]
    out = [None] * len(xs)
    if idx:
        vals = np.array([xs[i] for i in idx], dtype=np.float64).astype(np.float32).tolist()
        for i, v in zip(idx, vals):
            out[i] = v
    return out


def columns_to_retain_blocking(settings) -> List[str]:
    """Column order of the comparison frame (blocking.py:38-57)."""
    cols = {settings["unique_id_column_name"]: None}
    for c in settings["comparison_columns"]:
        if "col_name" in c:
            cols[c["col_name"]] = None
        for c2 in c.get("custom_columns_used", []):
            cols[c2] = None
    for c in settings["additional_columns_to_retain"]:
        cols[c] = None
    return list(cols)


def schema_of(tables) -> Schema:
    """Each column's form (str / num) over the input tables (the first table's wins)."""
    forms = {}
    for t in reversed(tables):
        for c in t.columns:
            forms[c] = T.natural_form(t[c])
    return Schema(forms)


def string_columns_read(settings, tables) -> List[str]:
    """Input string columns the settings' comparison program reads as bare operands, in program order: its
    derived columns (`lower(first_name)`, evaluated at ingest and uploaded under that name) and numeric
    columns left out.  Compiles on the host only."""
    prog = compile_comparisons(settings, schema_of(tables))
    out = []
    for name, form in prog.columns:
        if form == "str" and name not in prog.derived and name in tables[0].columns and name not in out:
            out.append(name)
    return out


class Job:
    """Record tables + pairs + codes living on one GPU.

    `inputs` are the tables as given (input row order).  Their columns go to the device once as
    Arrow buffers (spk_raw_*); blocking keys, dictionary ids, unique-id ranks and the clustering of
    the rows by the first rule's key are computed there (spk_key_build, spk_rank_from_raw,
    spk_cluster).  Device row i of side s is input row perm[s][i]; `tables` are the inputs in that
    order (materialised on demand, for output columns and checks)."""

    def __init__(self, link_type: str, tables: List[pd.DataFrame], unique_id_col: str, device: int,
                 shard=(0, 1), cluster: bool = True, replicate: bool = False, prefetch=None):
        self.link_type = link_type
        self.cluster = cluster
        self.inputs = [t.reset_index(drop=True) for t in tables]
        self.perm = [None] * len(self.inputs)
        self._views = {}
        self._host_cols = {}
        self.uid = unique_id_col
        self.device = device
        self.shard, self.n_shards = shard
        self.ctx = N.Context(device)
        self.ctx.set_link_type(N.LINK_TYPES[link_type])
        self.schema = schema_of(self.inputs)
        self._col_index = {}
        self._raw = {}
        self._next_raw = 0  # raw-column ids only go up: a released id is never handed out again
        self._prefetch = {}  # (side, name, "utf8") -> future of a background upload (prefetch_strings)
        self._prefetch_pool = None
        for side, t in enumerate(self.inputs):
            self.ctx.table_create(side, len(t), 8)
        self.n_pairs = 0
        self.n_candidates = 0
        self._pairs_host = None
        self.codes_token = None
        self.code_meta = None
        self.timings = {}
        self.force_reduce = False  # tests: the multi-GPU EM path (histogram -> all-reduce -> finalize) at one rank
        # ranks of a sharded job upload 1/G of each string column and all-gather the rest (tests: force it at
        # one rank with force_replicate)
        self.force_replicate = bool(replicate)
        self.replicate_ingest = self.reduces_across_ranks() or self.force_replicate
        if prefetch:
            self.prefetch_strings(prefetch)
        self._set_rank()

    @classmethod
    def from_gamma_table(cls, df: pd.DataFrame, gamma_names, device: int):
        """A job whose comparison vectors are given (the reference's iterate() on a gamma table)."""
        job = cls("dedupe_only", [pd.DataFrame({"_row": np.zeros(0, dtype=np.int64)})], "_row", device)
        job.passthrough = df.reset_index(drop=True)
        job.n_pairs = len(df)
        return job

    # ---- tables --------------------------------------------------------------------------------
    @property
    def tables(self) -> List[pd.DataFrame]:
        """The input tables in device row order (pair rows index these)."""
        return [self.table_view(s) for s in range(len(self.inputs))]

    def table_view(self, side: int) -> pd.DataFrame:
        if self.perm[side] is None:
            return self.inputs[side]
        if side not in self._views:
            self._views[side] = self.inputs[side].take(self.perm[side]).reset_index(drop=True)
        return self._views[side]

    def r_side(self) -> int:
        return 1 if self.link_type == "link_only" else 0

    def r_table(self) -> pd.DataFrame:
        return self.table_view(self.r_side())

    def host_values(self, side: int, name: str) -> np.ndarray:
        """Column `name` of side `side` as a numpy array in device row order."""
        key = (side, name)
        if key not in self._host_cols:
            col = self.inputs[side][name]
            if isinstance(col.dtype, pd.api.extensions.ExtensionDtype):  # Arrow / nullable: NULL as None
                v = col.to_numpy(dtype=object, na_value=None)
            else:
                v = col.to_numpy()
            self._host_cols[key] = v if self.perm[side] is None else v[self.perm[side]]
        return self._host_cols[key]

    def _new_raw(self) -> int:
        """A fresh raw-column index.  Released columns leave _raw (release_raw_strings), so len(_raw) could
        name an index a live column still holds (spk_raw_* replaces whatever is there): ids come from a
        counter instead."""
        rid = self._next_raw
        self._next_raw += 1
        return rid

    def prefetch_strings(self, names) -> int:
        """Start copying input string columns to the device in a background host thread (a torch stream of
        its own), so that the host-to-device upload of comparison-only columns -- first-touch pageable copies
        at ~7-11 GB/s, 1.6 s of the 100M-record share's job -- overlaps the unique-id ranks,
        the blocking keys and the clustering, which do not need them.  raw_utf8() adopts a prefetched column
        with one device-to-device copy (spk_raw_utf8_arrow, on_device = 1).  Only Arrow-backed columns of a
        job that uploads its own rows (not a replicated-ingest rank) are prefetched; returns how many."""
        if self.replicate_ingest:
            return 0
        import concurrent.futures as cf
        sides = [0, 1] if self.link_type == "link_only" else [0]
        todo = []
        for side in sides:
            for name in names:
                key = (side, name, "utf8")
                if key in self._raw or key in self._prefetch or name not in self.inputs[side].columns:
                    continue
                chunks = T.arrow_large_utf8_chunks(self.inputs[side][name])
                if chunks is not None:
                    todo.append((key, chunks))
        if not todo:
            return 0
        if self._prefetch_pool is None:
            self._prefetch_pool = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="spk-prefetch")
        for key, chunks in todo:
            self._prefetch[key] = self._prefetch_pool.submit(_upload_utf8_chunks, chunks, self.device)
        return len(todo)

    def drop_prefetch(self, keep=()):
        """Drop the background uploads of columns not in `keep` (no comparison program adopted them: e.g. a
        program that changed after blocking); their staging tensors go back to the device."""
        drop = [k for k in self._prefetch if k[1] not in keep]
        for key in drop:
            fut = self._prefetch.pop(key)
            if not fut.cancel():
                fut.result()  # running or done: wait, then let its tensors go
        if drop and not self._prefetch:
            import torch
            torch.cuda.empty_cache()
        return len(drop)

    def raw_utf8(self, side: int, name: str) -> int:
        """Raw string column (input row order) on the device, uploaded once.  Arrow columns hand over their
        buffers as they are (no host copy; rebasing and the validity bitmap are handled on the device).  A
        rank of a sharded job (replicate_ingest) uploads only its slice of the rows and gets the rest from
        the other ranks (distributed.allgather_utf8_rows): one host upload of the records per job, not per
        rank."""
        key = (side, name, "utf8")
        if key not in self._raw and key in self._prefetch:
            import time
            t0 = time.perf_counter()
            n, off, data, valid = self._prefetch.pop(key).result()
            t1 = time.perf_counter()
            rid = self._new_raw()
            self.ctx.raw_utf8_device(rid, n, off.data_ptr(), data.data_ptr(), valid.data_ptr())
            self.ctx.sync()
            del off, data, valid
            self._raw[key] = rid
            self.timings["prefetch_wait_s"] = self.timings.get("prefetch_wait_s", 0.0) + (t1 - t0)
            if not self._prefetch:
                import torch
                torch.cuda.empty_cache()  # the staging tensors: back to the device for the library's allocations
            return rid
        if key not in self._raw:
            rid = self._new_raw()
            chunks = None if self.replicate_ingest else T.arrow_large_utf8_chunks(self.inputs[side][name])
            if chunks is not None and len(chunks) > 1:
                # a chunked column: each chunk's buffers as they are, no host-side combine copy
                self.ctx.raw_utf8_arrow_chunks(rid, [T.arrow_views(c) for c in chunks], [len(c) for c in chunks])
                self._raw[key] = rid
                return rid
            arr = T.arrow_large_utf8(self.inputs[side][name])
            if arr is not None and self.replicate_ingest:
                n, off, data, valid, on_dev = D.allgather_utf8_rows(arr, force=self.force_replicate)
                if on_dev:
                    import torch
                    self.ctx.raw_utf8_device(rid, n, off.data_ptr(), data.data_ptr(), valid.data_ptr())
                    self.ctx.sync()
                    # the gathered tensors (about the column's size, x2 at the peak) go back to the device for the
                    # library's own allocations instead of staying reserved by torch's caching allocator
                    del off, data, valid
                    torch.cuda.empty_cache()
                else:
                    self.ctx.raw_utf8_arrow(rid, n, off, data, valid, -1)
            elif arr is not None:
                off, data, bitmap, bit0 = T.arrow_views(arr)
                self.ctx.raw_utf8_arrow(rid, len(arr), off, data, bitmap, bit0)
            else:
                off, data, valid = T.arrow_utf8(self.inputs[side][name])
                self.ctx.raw_utf8(rid, off, data, valid)
            self._raw[key] = rid
        return self._raw[key]

    def raw_i64(self, key, values, valid) -> int:
        if key not in self._raw:
            rid = self._new_raw()
            self.ctx.raw_i64(rid, values, valid)
            self._raw[key] = rid
        return self._raw[key]

    def _set_rank(self):
        """Order rank of every row for the link-type predicate (blocking.py:136, :139).  A NULL
        unique id never satisfies `l.uid < r.uid`; its rows get the last rank of their source and
        the kernel drops their same-source pairs (spk_table_set_rank_null).  Integer ids are ranked
        on the device (spk_rank_from_raw); others in Spark's order on the host."""
        if self.link_type == "link_only":
            return
        t = self.inputs[0]
        if self.uid not in t.columns:
            raise ValueError(f"unique_id_column_name {self.uid!r} is not a column of the input data")
        col = t[self.uid]
        right_from = -1
        if self.link_type == "link_and_dedupe":
            src = (t["_source_table"].to_numpy() == "right")
            right_from = int(np.argmax(src)) if src.any() else len(t)
            assert src[right_from:].all(), "link_and_dedupe: the right table's rows follow the left table's"
        if pd.api.types.is_integer_dtype(col.dtype) and not pd.api.types.is_bool_dtype(col.dtype):
            vals, valid = T.numeric_key_bits(col)
            self.ctx.rank_from_raw(self.raw_i64(("uid",), vals, valid), right_from)
            return
        uid_rank, nulls = T.dense_rank(col.tolist())
        n_distinct = int(uid_rank[~nulls].max()) + 1 if (~nulls).any() else 0
        div = n_distinct + 1  # r in [0, n_distinct) for ids, n_distinct for NULL
        r = np.where(nulls, n_distinct, uid_rank)
        rank = r
        if self.link_type == "link_and_dedupe":
            rank = (np.arange(len(t)) >= right_from).astype(np.int64) * div + r
        self.ctx.table_set_rank(0, np.asarray(rank, dtype=np.int64))
        self.ctx.table_set_rank_null(0, div if nulls.any() else 0)

    def column_index(self, name: str, form: str) -> int:
        key = (name, form)
        if key in self._col_index:
            return self._col_index[key]
        idx = len(self._col_index)
        sides = [0, 1] if self.link_type == "link_only" else [0]
        for side in sides:
            if name not in self.inputs[side].columns:
                raise ValueError(f"column {name!r} is missing from input table {side}")
        if form == "str":
            # decoded on the device through the row permutation; dictionary ids computed there, in one
            # id space for both sides (string equality = one integer compare)
            import time
            t0 = time.perf_counter()
            raws = [self.raw_utf8(side, name) for side in sides]
            t1 = time.perf_counter()
            self.ctx.table_add_raw_utf8(idx, raws[0], raws[1] if len(raws) > 1 else -1)
            t2 = time.perf_counter()
            self.timings["raw_upload_s"] = self.timings.get("raw_upload_s", 0.0) + (t1 - t0)
            self.timings["column_encode_s"] = self.timings.get("column_encode_s", 0.0) + (t2 - t1)
        else:
            for side in sides:
                vals, valid = T.encode_float64(self.inputs[side][name])
                if self.perm[side] is not None:
                    vals, valid = vals[self.perm[side]], valid[self.perm[side]]
                self.ctx.table_add_float64(side, idx, vals, valid)
        self._col_index[key] = idx
        return idx

    def add_derived(self, name: str, node):
        """A derived column (derived.py: a Spark built-in over one record's columns in a case_expression),
        evaluated once per row of each input table at ingest and added to the inputs under its canonical
        name, so it goes to the device and into the comparison programs like an input column."""
        from . import derived as D
        sides = [0, 1] if self.link_type == "link_only" else [0]
        form = D.form_of(node, self.schema.form)
        for side in sides:
            if name in self.inputs[side].columns:
                continue
            self.inputs[side][name] = D.evaluate(node, self.inputs[side], form)
            self._views.pop(side, None)
        self.schema.forms[name] = form
        self.schema._lower[name.lower()] = name

    # ---- blocking ----------------------------------------------------------------------------------
    def _key_values(self, t: pd.DataFrame, kexpr):
        s = t[kexpr.column]
        if not kexpr.transforms:
            return pd.Series([None if T.is_null_scalar(v) else v for v in s.tolist()], dtype=object)
        out = []
        for v in s.tolist():
            if T.is_null_scalar(v):
                out.append(None)
                continue
            x = T.spark_str(v)
            for tr in kexpr.transforms:
                if tr[0] == "substr":
                    x = T.spark_substr(x, tr[1], tr[2])
                elif tr[0] == "lower":
                    x = x.lower()
                elif tr[0] == "upper":
                    x = x.upper()
                elif tr[0] == "trim":
                    x = x.strip(" ")
            out.append(x)
        return pd.Series(out, dtype=object)

    @staticmethod
    def _substr_of(kexpr):
        """(start, len) of a key expression that is a column or one substr of it; None otherwise."""
        if not kexpr.transforms:
            return (0, -1)
        if len(kexpr.transforms) == 1 and kexpr.transforms[0][0] == "substr" and kexpr.transforms[0][2] >= 0:
            return (int(kexpr.transforms[0][1]), int(min(kexpr.transforms[0][2], 2 ** 31 - 1)))
        return None

    def _term(self, r, i, lexpr, rexpr, symmetric):
        """spk_key_term of one `l.a = r.b` term.  String columns (optionally under one substr) and plain
        numeric columns are keyed on the device from their raw buffers; other expressions (lower /
        upper / trim, mixed types) get their key ids on the host, uploaded as an int64 raw column."""
        s0, s1 = 0, self.r_side()
        fl, fr = self.schema.form(lexpr.column), self.schema.form(rexpr.column)
        sl, sr = self._substr_of(lexpr), self._substr_of(rexpr)
        same_raw = symmetric and self.link_type != "link_only"
        if fl == fr == "str" and sl is not None and sr is not None:
            raw_l = self.raw_utf8(s0, lexpr.column)
            raw_r = -1 if same_raw else self.raw_utf8(s1, rexpr.column)
            return (raw_l, raw_r, sl[0], sl[1], sr[0], sr[1])
        cl, cr = self.inputs[s0][lexpr.column], self.inputs[s1][rexpr.column]
        if fl == fr == "num" and not lexpr.transforms and not rexpr.transforms:
            ints = all(pd.api.types.is_integer_dtype(c.dtype) and not pd.api.types.is_bool_dtype(c.dtype)
                       for c in (cl, cr))
            conv = (lambda c: T.numeric_key_bits(c)) if ints else \
                (lambda c: T.numeric_key_bits(pd.to_numeric(c, errors="coerce").astype(np.float64)))
            raw_l = self.raw_i64((s0, lexpr.column, "num", ints), *conv(cl))
            raw_r = -1 if same_raw else self.raw_i64((s1, rexpr.column, "num", ints), *conv(cr))
            return (raw_l, raw_r, 0, -1, 0, -1)
        kl = self._key_values(self.inputs[s0], lexpr)
        kr = kl if same_raw else self._key_values(self.inputs[s1], rexpr)
        codes, _ = T.factorize_joint([kl, kr])
        raw_l = self.raw_i64(("key", r, i, "l"), codes[0], codes[0] >= 0)
        raw_r = -1 if same_raw else self.raw_i64(("key", r, i, "r"), codes[1], codes[1] >= 0)
        return (raw_l, raw_r, 0, -1, 0, -1)

    def block(self, rules: List[str]):
        import time
        t_start = time.perf_counter()
        n0, nr = len(self.inputs[0]), len(self.inputs[self.r_side()])
        symmetric = []
        if not rules:
            self.ctx.table_set_key(0, 0, 0, np.zeros(n0, dtype=np.int64))
            self.ctx.table_set_key(self.r_side(), 0, 1, np.zeros(nr, dtype=np.int64))
            symmetric = [1]
        for r, text in enumerate(rules):
            spec = compile_rule(text, self.schema)
            terms = [self._term(r, i, lexpr, rexpr, lexpr == rexpr) for i, (lexpr, rexpr) in enumerate(spec.terms)]
            self.ctx.key_build(r, terms)
            symmetric.append(1 if spec.symmetric else 0)
        if rules and self.cluster:
            # rows of a block become contiguous: the comparison pass reads a block's records from a few
            # cache lines.  The pair set and its ordinal order do not change (blocking sorts by key, rank).
            p0, p1 = self.ctx.cluster(n0, len(self.inputs[1]) if self.link_type == "link_only" else None)
            self.perm = [p0] + ([p1] if p1 is not None else [])
            self._views, self._host_cols, self._col_index, self._prog_cache = {}, {}, {}, {}
        t_keys = time.perf_counter()
        self.n_pairs, self.n_candidates = self.ctx.block(N.LINK_TYPES[self.link_type], symmetric, self.shard,
                                                         self.n_shards)
        self.timings["block_keys_s"] = t_keys - t_start
        self.timings["block_pairs_s"] = time.perf_counter() - t_keys
        self._pairs_host = None
        self.codes_token = None
        return self.n_pairs

    def load_pairs(self, rows_l, rows_r):
        self.ctx.pairs_load(rows_l, rows_r)
        self.n_pairs = len(rows_l)
        self._pairs_host = (np.asarray(rows_l, dtype=np.int32), np.asarray(rows_r, dtype=np.int32))
        self.codes_token = None

    def pair_rows(self):
        if self._pairs_host is None:
            self._pairs_host = self.ctx.pairs_copy(0, self.n_pairs)
        return self._pairs_host

    # ---- comparison vectors -----------------------------------------------------------------------
    def _compiled(self, settings):
        """The comparison program and its native buffers, compiled once per distinct comparison_columns."""
        # the program depends only on each column's name, level count and CASE text
        key = tuple((c.get("col_name"), c.get("custom_name"), c.get("num_levels"), c.get("case_expression"))
                    for c in settings["comparison_columns"])
        cache = self.__dict__.setdefault("_prog_cache", {})
        if key not in cache:
            prog = compile_comparisons(settings, self.schema)
            for name, node in prog.derived.items():
                self.add_derived(name, node)
            index = {k: self.column_index(*k) for k in prog.columns}
            if self._prefetch:
                self.drop_prefetch(keep={name for name, _ in prog.columns})
            lit_off, lit_bytes = prog.literal_buffers()
            args = N.Context.gammas_args(prog.programs, prog.when_first, prog.when_n, prog.when_level, prog.instrs,
                                         prog.native_operands(index), lit_off, lit_bytes)
            cache[key] = (prog, args)
        return cache[key]

    def release_raw_strings(self):
        """Free the device copies of the input string columns once the comparison columns are decoded from
        them and the blocking keys built (at 100M records ~20 GB of UTF-8 bytes and offsets); a later
        block() or a new comparison column uploads what it needs again."""
        for key in [k for k in self._raw if len(k) == 3 and k[2] == "utf8"]:
            self.ctx.raw_release(self._raw.pop(key))

    def gammas(self, settings, token=None) -> CompiledComparisons:
        prog, args = self._compiled(settings)
        if self.n_pairs > 0:
            self.release_raw_strings()
        self.ctx.gammas_native(args)
        self.codes_token = token if token is not None else object()
        self.code_meta = (prog.gamma_names, prog.n_levels)
        return prog

    def load_gammas(self, gamma_names, n_levels, gammas: np.ndarray, token=None):
        self.ctx.gammas_load(n_levels, gammas)
        self.n_pairs = gammas.shape[0]
        self.codes_token = token if token is not None else object()
        self.code_meta = (list(gamma_names), list(n_levels))

    def gammas_host(self):
        names, levels = self.code_meta
        return self.ctx.gammas_copy(len(names), 0, self.n_pairs)

    # ---- EM -------------------------------------------------------------------------------------------
    def reduces_across_ranks(self) -> bool:
        """True when this job holds one rank's shard of a pair set split over the process group:
        its sufficient statistics (EM histogram, tf tables) must be summed over ranks.  A job whose
        pairs are not sharded (a gamma table handed to iterate(), or a test's explicit shard without
        a process group) keeps its statistics local."""
        rank, world = distributed_shard()
        return world > 1 and self.n_shards == world and self.shard == rank

    @staticmethod
    def flat_tables(level_probs):
        m = [quantise(p) for mk, _ in level_probs for p in mk]
        u = [quantise(p) for _, uk in level_probs for p in uk]
        return np.array(m, dtype=np.float64), np.array(u, dtype=np.float64)

    def em_stats(self, lam, level_probs):
        """One fused E+M pass over every pair's comparison vector; returns the M-step statistics."""
        names, n_levels = self.code_meta
        m, u = self.flat_tables(level_probs)
        lam_d, one_minus = float(lam), float(1 - lam)
        n_stats = N_HEAD + 4 * sum(L + 1 for L in n_levels)
        if self.reduces_across_ranks() or self.force_reduce:
            import torch
            hist = self._device_hist()
            self.ctx.em_histogram(hist.data_ptr())  # zeroes, fills and synchronises its stream
            D.allreduce_histogram_(hist, force=self.force_reduce)
            torch.cuda.synchronize(self.device)
            return self.ctx.em_finalize(hist.data_ptr(), lam_d, one_minus, m, u, n_stats)
        return self.ctx.em_iteration(lam_d, one_minus, m, u, n_stats)

    def _device_hist(self):
        import torch
        n_pat = self.ctx.n_patterns()
        hist = getattr(self, "_hist_dev", None)
        if hist is None or hist.numel() != n_pat:
            hist = torch.empty(n_pat, dtype=torch.int64, device=f"cuda:{self.device}")
            # the buffer is written on the context's stream: torch's allocation work must be done
            torch.cuda.synchronize(self.device)
            self._hist_dev = hist
        return hist

    def _collective_stream(self):
        """The torch stream this job's context runs on once its EM exchange is stream-ordered (RCCL):
        histogram -> all-reduce -> finalize are then queued back to back with no host synchronisation."""
        import torch
        s = getattr(self, "_dist_stream", None)
        if s is None:
            s = torch.cuda.Stream(device=self.device)
            torch.cuda.synchronize(self.device)
            self.ctx.sync()
            self.ctx.set_stream(s.cuda_stream)
            self._dist_stream = s
        return s

    def em_start(self, lam, level_probs):
        """em_stats in two halves: enqueue the iteration now, collect its statistics with em_wait().  On
        one GPU the launch and the statistics readback are asynchronous (spk_em_iteration_start), so the
        next comparison pass can be queued and the host M-step computed while the device works.  With a
        cross-rank reduction over RCCL the histogram, the all-reduce and the finalize are queued on one
        stream (spk_em_histogram_async, dist.all_reduce, spk_em_finalize_start); under gloo (host staging)
        the iteration runs synchronously here."""
        names, n_levels = self.code_meta
        self._em_n_stats = N_HEAD + 4 * sum(L + 1 for L in n_levels)
        self._em_done = None
        if self.reduces_across_ranks() or self.force_reduce:
            if not D.stream_ordered_reduce(self.device):
                self._em_done = self.em_stats(lam, level_probs)
                return
            import torch
            m, u = self.flat_tables(level_probs)
            s = self._collective_stream()
            hist = self._device_hist()
            self.ctx.em_histogram_async(hist.data_ptr())
            with torch.cuda.stream(s):
                D.allreduce_histogram_(hist, force=self.force_reduce)
            self.ctx.em_finalize_start(hist.data_ptr(), float(lam), float(1 - lam), m, u, self._em_n_stats)
            return
        m, u = self.flat_tables(level_probs)
        self.ctx.em_iteration_start(float(lam), float(1 - lam), m, u, self._em_n_stats)

    def em_wait(self):
        if self._em_done is not None:
            out, self._em_done = self._em_done, None
            return out
        return self.ctx.em_iteration_wait(self._em_n_stats)

    def log_likelihood(self, lam, level_probs):
        """Σ over pairs of ln(λ·Πm + (1-λ)·Πu) (expectation_step.py:224-272); None if every term is NULL."""
        stats = self.em_stats(lam, level_probs)
        return float(stats[3]) if stats[4] > 0 else None

    def score(self, lam, level_probs, want_host=True):
        m, u = self.flat_tables(level_probs)
        return self.ctx.score(float(lam), float(1 - lam), m, u, 0, self.n_pairs, want_host)


def _upload_utf8_chunks(chunks, device: int):
    """Background half of Job.prefetch_strings: the Arrow chunks of one string column as device tensors in
    the form spk_raw_utf8_arrow(on_device = 1) takes -- int64 offsets from 0 [n + 1], the bytes, one
    validity byte per row -- copied on a torch stream of this thread's own (the copies release the GIL)."""
    import torch
    dev = torch.device(f"cuda:{device}")
    n = sum(len(c) for c in chunks)
    views = [T.arrow_views(c) for c in chunks]
    nbytes = sum(int(v[0][-1] - v[0][0]) for v in views)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        data = torch.empty(nbytes + 1, dtype=torch.uint8, device=dev)
        valid = torch.empty(n + 1, dtype=torch.uint8, device=dev)
        r0, b0 = 0, 0
        for c, (o, d, bitmap, bit0) in zip(chunks, views):
            rows = len(c)
            lo, hi = int(o[0]), int(o[-1])
            if hi > lo:
                data[b0:b0 + hi - lo].copy_(torch.from_numpy(d[lo:hi]))
            oc = torch.from_numpy(np.ascontiguousarray(o)).to(dev)
            off[r0:r0 + rows + 1] = oc - (lo - b0)
            if bitmap is None:
                valid[r0:r0 + rows].fill_(1)
            else:
                bits = np.unpackbits(bitmap, bitorder="little")[bit0: bit0 + rows]
                valid[r0:r0 + rows].copy_(torch.from_numpy(bits))
            r0 += rows
            b0 += hi - lo
        data[nbytes:].fill_(0)
        valid[n:].fill_(0)
    stream.synchronize()
    return n, off, data, valid


def _sum_lr(xs):
    acc = 0.0
    for x in xs:
        acc += x
    return acc


def m_step_rows(stats, gamma_names, n_levels):
    """λ and the collected π rows (maximisation_step.py:16-90) from the device statistics,
    with Spark's NULL and float32 semantics."""
    stats = stats.tolist() if isinstance(stats, np.ndarray) else [float(x) for x in stats]
    S, rows, nn = stats[0], stats[1], stats[2]
    new_lambda = f32(S / rows) if (rows > 0 and nn > 0) else None
    out = []
    off = N_HEAD
    for name, L in zip(gamma_names, n_levels):
        slots = [stats[off + 4 * i: off + 4 * i + 4] for i in range(L + 1)]
        off += 4 * (L + 1)
        observed = slots[1:]
        # the denominators sum the observed levels in level order, as numpy's pairwise sum did for
        # these short vectors (<= 8 terms: plain left-to-right addition)
        den_nonnull = sum(o[1] for o in observed) > 0
        den_m, den_u = _sum_lr([o[2] for o in observed]), _sum_lr([o[3] for o in observed])
        for v in range(-1, L):
            r, nnv, sm, su = slots[v + 1]
            if r == 0:
                continue
            if nnv == 0 or not den_nonnull:
                pm = pu = None
            else:
                pm = sm / den_m if den_m != 0 else None
                pu = su / den_u if den_u != 0 else None
            out.append({"gamma_value": v, "new_probability_match": pm, "new_probability_non_match": pu,
                        "gamma_col": name})
    # Spark's float cast of every ratio, in one conversion
    cast = f32_many([x for r in out for x in (r["new_probability_match"], r["new_probability_non_match"])])
    for i, r in enumerate(out):
        r["new_probability_match"], r["new_probability_non_match"] = cast[2 * i], cast[2 * i + 1]
    return new_lambda, out
