"""Device-resident, lazily materialised frames returned by the stage functions.

They stand where the reference returns Spark DataFrames (blocking.py:162, gammas.py:93,
expectation_step.py:26, term_frequencies.py:123) and offer the slice of that surface the
pipeline and its users need: `toPandas()`, `count()`, `columns`, `persist()` / `cache()` /
`unpersist()`, `createOrReplaceTempView()`.  Pairs, comparison codes and scores stay on the
GPU; `toPandas()` copies them back and gathers the retained input columns with the
reference's column names and order.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import pandas as pd


class SplinkDataFrame:
    """Common surface of the lazily evaluated frames."""

    def toPandas(self) -> pd.DataFrame:  # noqa: N802 (Spark name)
        raise NotImplementedError

    def to_pandas(self) -> pd.DataFrame:
        return self.toPandas()

    def count(self) -> int:
        return int(self.job.n_pairs)

    def __len__(self):
        return self.count()

    @property
    def columns(self):
        return list(self._column_order())

    def persist(self, *args, **kwargs):
        return self

    cache = persist

    def unpersist(self, *args, **kwargs):
        return self

    def createOrReplaceTempView(self, name):  # noqa: N802 (Spark name)
        return None


def _add_lr(cols: "OrderedDict", name: str):
    cols[name + "_l"] = None
    cols[name + "_r"] = None


def comparison_column_order(settings, link_type):
    """blocking.py:18-36 + _get_columns_to_retain_blocking, with _source_table for link_and_dedupe."""
    from .engine import columns_to_retain_blocking
    cols = columns_to_retain_blocking(settings)
    if link_type == "link_and_dedupe":
        cols = cols + ["_source_table"]
    out = OrderedDict()
    for c in cols:
        _add_lr(out, c)
    return list(out)


def gamma_column_order(settings):
    """gammas.py:25-62."""
    out = OrderedDict()
    _add_lr(out, settings["unique_id_column_name"])
    for col in settings["comparison_columns"]:
        if "col_name" in col:
            name = col["col_name"]
            if settings["retain_matching_columns"] or col["term_frequency_adjustments"]:
                _add_lr(out, name)
            out["gamma_" + name] = None
        if "custom_name" in col:
            if settings["retain_matching_columns"]:
                for c2 in col["custom_columns_used"]:
                    _add_lr(out, c2)
            out["gamma_" + col["custom_name"]] = None
    if settings["link_type"] == "link_and_dedupe":
        _add_lr(out, "_source_table")
    for c in settings["additional_columns_to_retain"]:
        _add_lr(out, c)
    return list(out)


def df_e_column_order(settings, tf_adj_cols=False):
    """expectation_step.py:128-165."""
    out = OrderedDict()
    _add_lr(out, settings["unique_id_column_name"])
    for col in settings["comparison_columns"]:
        if "col_name" in col:
            name = col["col_name"]
            if settings["retain_matching_columns"] or col["term_frequency_adjustments"]:
                _add_lr(out, name)
            out["gamma_" + name] = None
        if "custom_name" in col:
            name = col["custom_name"]
            if settings["retain_matching_columns"]:
                for c2 in col["custom_columns_used"]:
                    _add_lr(out, c2)
            out["gamma_" + name] = None
        if settings["retain_intermediate_calculation_columns"]:
            out[f"prob_gamma_{name}_non_match"] = None
            out[f"prob_gamma_{name}_match"] = None
            if tf_adj_cols and col.get("term_frequency_adjustments"):
                out[name + "_adj"] = None
    if settings["link_type"] == "link_and_dedupe":
        _add_lr(out, "_source_table")
    for c in settings["additional_columns_to_retain"]:
        _add_lr(out, c)
    return list(out)


class _HostColumns:
    """Gathers `<col>_l` / `<col>_r` values for the job's pairs from the host input tables."""

    def __init__(self, job):
        self.job = job
        self._cache = {}

    def get(self, name):
        if name in self._cache:
            return self._cache[name]
        job = self.job
        if getattr(job, "passthrough", None) is not None:
            df = job.passthrough
            if name not in df.columns:
                raise KeyError(name)
            v = df[name].to_numpy()
        else:
            base, side = name[:-2], name[-2:]
            rows_l, rows_r = job.pair_rows()
            s = 0 if side == "_l" else job.r_side()
            if base not in job.inputs[s].columns:
                raise KeyError(name)
            v = job.host_values(s, base)[rows_l if side == "_l" else rows_r]
        self._cache[name] = v
        return v


class ComparisonFrame(SplinkDataFrame):
    """Candidate pairs (block_using_rules)."""

    def __init__(self, job, settings):
        self.job = job
        self.settings = settings

    def _column_order(self):
        return comparison_column_order(self.settings, self.job.link_type)

    def toPandas(self):
        host = _HostColumns(self.job)
        return pd.DataFrame({c: host.get(c) for c in self._column_order()})


class GammaFrame(SplinkDataFrame):
    """Comparison vectors (add_gammas): packed codes on the device."""

    def __init__(self, job, settings, program=None, gammas=None):
        self.job = job
        self.settings = settings
        self.program = program
        self._host_gammas = gammas
        self.token = object()
        if gammas is None:
            job.gammas(settings, token=self.token)
        else:
            names, levels = program
            job.load_gammas(names, levels, gammas, token=self.token)

    def ensure_codes(self):
        """Re-install this frame's codes if another frame of the same job replaced them."""
        if self.job.codes_token is not self.token:
            if self._host_gammas is None:
                self.job.gammas(self.settings, token=self.token)
            else:
                names, levels = self.program
                self.job.load_gammas(names, levels, self._host_gammas, token=self.token)

    @property
    def gamma_names(self):
        return self.job.code_meta[0]

    @property
    def n_levels(self):
        return self.job.code_meta[1]

    def gamma_matrix(self) -> np.ndarray:
        self.ensure_codes()
        return self.job.gammas_host()

    def _column_order(self):
        if getattr(self.job, "passthrough", None) is not None:
            return list(self.job.passthrough.columns)
        return gamma_column_order(self.settings)

    def _frame(self, order):
        host = _HostColumns(self.job)
        gam = self.gamma_matrix()
        gidx = {n: i for i, n in enumerate(self.gamma_names)}
        data = OrderedDict()
        for c in order:
            if c in gidx:
                data[c] = gam[:, gidx[c]].astype(np.int32)
            else:
                data[c] = host.get(c)
        return pd.DataFrame(data)

    def toPandas(self):
        return self._frame(self._column_order())


class ExpectationFrame(SplinkDataFrame):
    """E-step output (run_expectation_step): lazily scored with the parameters it was created with."""

    def __init__(self, gamma_frame: GammaFrame, settings, lam, level_probs):
        self.gammas = gamma_frame
        self.job = gamma_frame.job
        self.settings = settings
        self.lam = lam
        self.level_probs = [(list(m), list(u)) for m, u in level_probs]
        self._mp = None

    def match_probability(self) -> np.ndarray:
        if self._mp is None:
            self.gammas.ensure_codes()
            self._mp = self.job.score(self.lam, self.level_probs)
        return self._mp

    def _column_order(self):
        return ["match_probability"] + df_e_column_order(self.settings)

    def _prob_columns(self, gam):
        out = {}
        from .engine import quantise
        for k, name in enumerate(self.gammas.gamma_names):
            g = name[len("gamma_"):]
            m, u = self.level_probs[k]
            mt = np.array([1.0] + [quantise(p) for p in m])
            ut = np.array([1.0] + [quantise(p) for p in u])
            idx = gam[:, k].astype(np.int64) + 1
            out[f"prob_gamma_{g}_match"] = mt[idx]
            out[f"prob_gamma_{g}_non_match"] = ut[idx]
        return out

    def toPandas(self):
        order = self._column_order()
        mp = self.match_probability()
        self.gammas.ensure_codes()
        gam = self.job.gammas_host()
        gidx = {n: i for i, n in enumerate(self.gammas.gamma_names)}
        probs = self._prob_columns(gam)
        host = _HostColumns(self.job)
        data = OrderedDict()
        for c in order:
            if c == "match_probability":
                data[c] = mp
            elif c in gidx:
                data[c] = gam[:, gidx[c]].astype(np.int32)
            elif c in probs:
                data[c] = probs[c]
            else:
                data[c] = host.get(c)
        return pd.DataFrame(data)
