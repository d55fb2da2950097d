"""M-step (reference: splink/maximisation_step.py:94-117).

The reference groups df_e by the full comparison vector, then collects λ and every π row
cast to float32.  Here the fused E+M pass (spk_em_histogram + spk_em_finalize) streams the
comparison codes once on the GPU and returns the grouped sums; the float32 / NULL semantics
of the collected rows are applied in engine.m_step_rows, and the rows go to
Params._update_params exactly as the reference passes them.
"""
from .engine import m_step_rows
from .params import Params


def run_maximisation_step(df_e, params: Params, spark):
    df_e.gammas.ensure_codes()
    names, levels = df_e.gammas.gamma_names, df_e.gammas.n_levels
    stats = df_e.job.em_stats(df_e.lam, df_e.level_probs)
    new_lambda, rows = m_step_rows(stats, names, levels)
    params._update_params(new_lambda, rows)
