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


class Job:
    """Record tables + pairs + codes living on one GPU."""

    def __init__(self, link_type: str, tables: List[pd.DataFrame], unique_id_col: str, device: int,
                 shard=(0, 1), cluster: bool = True):
        self.link_type = link_type
        self.cluster = cluster
        self.tables = [t.reset_index(drop=True) for t in tables]
        self.uid = unique_id_col
        self.device = device
        self.shard, self.n_shards = shard
        self.ctx = N.Context(device)
        self.ctx.set_link_type(N.LINK_TYPES[link_type])
        forms = {}
        for t in reversed(self.tables):
            for c in t.columns:
                forms[c] = T.natural_form(t[c])
        self.schema = Schema(forms)
        self._col_index = {}
        for side, t in enumerate(self.tables):
            self.ctx.table_create(side, len(t), 8)
        self.n_pairs = 0
        self.n_candidates = 0
        self._pairs_host = None
        self.codes_token = None
        self.code_meta = None
        self._set_rank()

    @classmethod
    def from_gamma_table(cls, df: pd.DataFrame, gamma_names, device: int):
        """A job whose comparison vectors are given (the reference's iterate() on a gamma table)."""
        job = cls("dedupe_only", [pd.DataFrame({"_row": np.zeros(0, dtype=np.int64)})], "_row", device)
        job.passthrough = df.reset_index(drop=True)
        job.n_pairs = len(df)
        return job

    # ---- tables --------------------------------------------------------------------------------
    def r_table(self) -> pd.DataFrame:
        return self.tables[1] if self.link_type == "link_only" else self.tables[0]

    def _set_rank(self):
        """Order rank of every row for the link-type predicate (blocking.py:136, :139).  A NULL
        unique id never satisfies `l.uid < r.uid`; its rows get the last rank of their source and
        the kernel drops their same-source pairs (spk_table_set_rank_null)."""
        self._rank = None
        if self.link_type == "link_only":
            return
        t = self.tables[0]
        if self.uid not in t.columns:
            raise ValueError(f"unique_id_column_name {self.uid!r} is not a column of the input data")
        col = t[self.uid]
        if (pd.api.types.is_integer_dtype(col.dtype) and not pd.api.types.is_bool_dtype(col.dtype)
                and not col.isna().any()):
            uid_rank, nulls = T.dense_rank_array(col.to_numpy(dtype=np.int64))
        else:
            uid_rank, nulls = T.dense_rank(col.tolist())
        n_distinct = int(uid_rank[~nulls].max()) + 1 if (~nulls).any() else 0
        div = n_distinct + 1  # r in [0, n_distinct) for ids, n_distinct for NULL
        r = np.where(nulls, n_distinct, uid_rank)
        if self.link_type == "link_and_dedupe":
            src = (t["_source_table"].to_numpy() == "right").astype(np.int64)
            rank = src * div + r
        else:
            rank = r
        self._rank = np.asarray(rank, dtype=np.int64)
        self.ctx.table_set_rank(0, self._rank)
        self.ctx.table_set_rank_null(0, div if nulls.any() else 0)

    def column_index(self, name: str, form: str) -> int:
        key = (name, form)
        if key in self._col_index:
            return self._col_index[key]
        idx = len(self._col_index)
        sides = [0, 1] if self.link_type == "link_only" else [0]
        for side in sides:
            if name not in self.tables[side].columns:
                raise ValueError(f"column {name!r} is missing from input table {side}")
        ids = None
        if form == "str":
            # dictionary ids in one id space for both sides: string equality becomes one integer compare
            ids, _ = T.factorize_joint([pd.Series(T.to_strings(self.tables[s][name]), dtype=object) for s in sides])
        for i, side in enumerate(sides):
            t = self.tables[side]
            if form == "str":
                off, data, valid = T.encode_utf8(t[name])
                self.ctx.table_add_utf8(side, idx, off, data, valid, ids[i])
            else:
                vals, valid = T.encode_float64(t[name])
                self.ctx.table_add_float64(side, idx, vals, valid)
        self._col_index[key] = idx
        return idx

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

    def _cluster(self, rule_keys):
        """Reorder the record tables by the first rule's blocking key (then rank), so a block's
        rows are contiguous on the device: the comparison pass reads a block's records from a few
        cache lines instead of one random line per row.  Pair rows then index the reordered tables;
        the pair set and its ordinal order do not change (blocking sorts by key and rank anyway)."""
        key_l, key_r = rule_keys[0]
        sides = [(0, key_l)] + ([(1, key_r)] if self.link_type == "link_only" else [])
        perms = {}
        for side, key in sides:
            n = len(self.tables[side])
            nulls_last = np.where(key < 0, np.iinfo(np.int64).max, key)
            rank = self._rank if (side == 0 and self._rank is not None) else np.arange(n, dtype=np.int64)
            perms[side] = np.lexsort((np.arange(n), rank, nulls_last))
        for side, perm in perms.items():
            self.tables[side] = self.tables[side].take(perm).reset_index(drop=True)
            self.ctx.table_create(side, len(self.tables[side]), 8)
        self._col_index = {}
        self._prog_cache = {}  # column uploads (and their indices) start again
        self._set_rank()
        p0 = perms[0]
        pr = perms.get(1, p0)
        return [(kl[p0], kr[pr]) for kl, kr in rule_keys]

    def block(self, rules: List[str]):
        t0, tr = self.tables[0], self.r_table()
        symmetric = []
        if not rules:
            self.ctx.table_set_key(0, 0, 0, np.zeros(len(t0), dtype=np.int64))
            side_r = 1 if self.link_type == "link_only" else 0
            self.ctx.table_set_key(side_r, 0, 1, np.zeros(len(tr), dtype=np.int64))
            symmetric = [1]
        rule_keys = []
        for text in rules:
            spec = compile_rule(text, self.schema)
            per_term = []
            for lexpr, rexpr in spec.terms:
                kl = self._key_values(t0, lexpr)
                # dedupe with a symmetric term (l.x = r.x): both sides read the same table and key
                kr = kl if (tr is t0 and lexpr == rexpr) else self._key_values(tr, rexpr)
                codes, _ = T.factorize_joint([kl, kr])
                per_term.append(codes)
            rule_keys.append(T.combine_codes(per_term))
            symmetric.append(1 if spec.symmetric else 0)
        if rule_keys and self.cluster:
            rule_keys = self._cluster(rule_keys)
        for r, (key_l, key_r) in enumerate(rule_keys):
            self.ctx.table_set_key(0, r, 0, key_l)
            self.ctx.table_set_key(1 if self.link_type == "link_only" else 0, r, 1, key_r)
        self.n_pairs, self.n_candidates = self.ctx.block(N.LINK_TYPES[self.link_type], symmetric, self.shard,
                                                         self.n_shards)
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
            index = {k: self.column_index(*k) for k in prog.columns}
            lit_off, lit_bytes = prog.literal_buffers()
            args = N.Context.gammas_args(prog.programs, prog.when_first, prog.when_n, prog.when_level, prog.instrs,
                                         prog.native_operands(index), lit_off, lit_bytes)
            cache[key] = (prog, args)
        return cache[key]

    def gammas(self, settings, token=None) -> CompiledComparisons:
        prog, args = self._compiled(settings)
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
        if self.reduces_across_ranks():
            import torch
            n_pat = self.ctx.n_patterns()
            hist = getattr(self, "_hist_dev", None)
            if hist is None or hist.numel() != n_pat:
                hist = torch.empty(n_pat, dtype=torch.int64, device=f"cuda:{self.device}")
                # the buffer is written on the context's stream: torch's allocation work must be done
                torch.cuda.synchronize(self.device)
                self._hist_dev = hist
            self.ctx.em_histogram(hist.data_ptr())  # zeroes, fills and synchronises its stream
            D.allreduce_histogram_(hist)
            torch.cuda.synchronize(self.device)
            return self.ctx.em_finalize(hist.data_ptr(), lam_d, one_minus, m, u, n_stats)
        self.ctx.em_histogram(0)
        return self.ctx.em_finalize(0, lam_d, one_minus, m, u, n_stats)

    def log_likelihood(self, lam, level_probs):
        """Σ over pairs of ln(λ·Πm + (1-λ)·Πu) (expectation_step.py:224-272); None if every term is NULL."""
        stats = self.em_stats(lam, level_probs)
        return float(stats[3]) if stats[4] > 0 else None

    def score(self, lam, level_probs, want_host=True):
        m, u = self.flat_tables(level_probs)
        return self.ctx.score(float(lam), float(1 - lam), m, u, 0, self.n_pairs, want_host)


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
