"""Term-frequency adjustment (reference: splink/term_frequencies.py:122-168).

Per tf column c: over pairs whose c_l and c_r are equal and non-NULL, the mean match
probability per value (adj_lambda, :49-65) is Bayes-combined with 1-λ; pairs without a
lookup value get 0.5 (:68-95); tf_adjusted_match_prob = bayes(mp, adj_c1, ...) (:98-117).
The per-value sums and the per-pair Bayes combination run on the GPU
(spk_tf_scales, spk_tf_accumulate_exact / spk_tf_apply): the sums are exact fixed-point accumulators
relative to each value's largest term, so ranks
holding shards of the pairs all-reduce them as integers and every run and rank count gives
bit-identical adjustments; the per-value lookup arithmetic is a handful of operations per value.
"""
import warnings
from collections import OrderedDict

import numpy as np
import pandas as pd

from . import _native as N
from . import distributed as D
from . import table as T
from .check_types import check_types
from .frames import ExpectationFrame, SplinkDataFrame, _HostColumns, df_e_column_order
from .params import Params


def _bayes_pair(a, b):
    """sql_gen_bayes_string([a, b]) (:21-46) for vectors a and a scalar b."""
    num = a * b
    den = num + (1.0 - a) * (1.0 - b)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = num / den
    out[den == 0] = np.nan
    return out


class TermFrequencyFrame(SplinkDataFrame):
    def __init__(self, df_e: ExpectationFrame, settings, tf_cols, tf_mp, adj, retain_adjustment_columns):
        self.df_e = df_e
        self.job = df_e.job
        self.settings = settings
        self.tf_cols = tf_cols
        self.tf_mp = tf_mp
        self.adj = adj
        self.retain = retain_adjustment_columns

    def _column_order(self):
        cols = ["tf_adjusted_match_prob", "match_probability"] + df_e_column_order(self.settings, tf_adj_cols=True)
        if not self.retain:
            cols = [c for c in cols if not (c.endswith("_adj") and c[:-4] in self.tf_cols)]
        return cols

    def toPandas(self):
        base = self.df_e.toPandas()
        data = OrderedDict()
        for c in self._column_order():
            if c == "tf_adjusted_match_prob":
                data[c] = self.tf_mp
            elif c.endswith("_adj") and c[:-4] in self.tf_cols:
                data[c] = self.adj[:, self.tf_cols.index(c[:-4])]
            else:
                data[c] = base[c].to_numpy()
        return pd.DataFrame(data)


@check_types
def make_adjustment_for_term_frequencies(df_e: object, params: Params, settings: dict, spark: object,
                                         retain_adjustment_columns: bool = False):
    tf_cols = [c["col_name"] for c in settings["comparison_columns"] if c["term_frequency_adjustments"] is True]
    if not tf_cols:
        warnings.warn("No term frequency adjustment columns are specified in your settings object.  "
                      "Returning original df")
        return df_e
    job = df_e.job
    df_e.gammas.ensure_codes()
    job.score(df_e.lam, df_e.level_probs, want_host=False)  # device mp for exactly this df_e
    one_minus = float(1 - params.params["λ"])
    # value ids: the device dictionary ids of the string column when the job decoded it on the device
    # (no host pass over the values), else a joint host factorisation
    dev_cols = [job._col_index.get((c, "str")) for c in tf_cols]
    on_device = all(i is not None for i in dev_cols)
    ids0_list, ids1_list, tables = [], [], []
    shared = job.reduces_across_ranks()  # the reference groups over ALL pairs (:49-65); ranks hold shards
    for c, col in zip(tf_cols, dev_cols):
        # two passes over the pairs: each value's scale (the exponent of its largest mp; MAX over ranks),
        # then the fixed-point sums relative to it (integer SUM over ranks): every rank ends with the
        # one-GPU result, and tiny match probabilities keep their relative precision
        if on_device:
            n_values = job.ctx.tf_column_values(col)
            scale = job.ctx.tf_scales_column(col, n_values)
        else:
            sides = (0, 1) if job.link_type == "link_only" else (0,)
            vals = [pd.Series([None if T.is_null_scalar(v) else v for v in job.host_values(s, c).tolist()],
                              dtype=object) for s in sides]
            codes, n_values = T.factorize_joint(vals)
            ids0 = codes[0]
            ids1 = codes[1] if len(codes) > 1 else codes[0]
            scale = job.ctx.tf_scales(n_values, ids0, ids1)
            ids0_list.append(ids0)
            ids1_list.append(ids1)
        if shared:
            D.allreduce_host_(scale, op="max")
        if on_device:
            limbs, counts = job.ctx.tf_accumulate_column_exact(col, n_values, scale)
        else:
            limbs, counts = job.ctx.tf_accumulate_exact(n_values, ids0, ids1, scale)
        if shared:
            # exact fixed-point sums and integer counts: the all-reduce gives every rank the one-GPU result
            D.allreduce_host_(limbs)
            D.allreduce_host_(counts)
        sums = N.tf_limbs_to_sum(limbs, scale)
        with np.errstate(invalid="ignore", divide="ignore"):
            adj_lambda = np.where(counts > 0, sums / np.maximum(counts, 1), np.nan)
        tables.append(_bayes_pair(adj_lambda, one_minus))
    if on_device:
        tf_mp, adj = job.ctx.tf_apply_columns(dev_cols, tables, 0, job.n_pairs, want_adj=True)
    else:
        tf_mp, adj = job.ctx.tf_apply(ids0_list, ids1_list, tables, 0, job.n_pairs, want_adj=True)
    return TermFrequencyFrame(df_e, settings, tf_cols, tf_mp, adj, retain_adjustment_columns)
