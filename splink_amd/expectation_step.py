"""E-step (reference: splink/expectation_step.py).

`run_expectation_step` returns a frame bound to the parameters current at the call, exactly
like the reference bakes λ / m / u into the SQL it generates (:167-221).  The per-pair
match probability -- (λ·m1·…·mK) / ((λ·m1·…·mK) + ((1-λ)·u1·…·uK)) with each m / u rendered as
`cast({p:.35f} as double)` -- is evaluated on the GPU (spk_score), or fused with the M-step
aggregate when the frame is handed to run_maximisation_step (spk_em_histogram/finalize).
"""
import logging

import numpy as np
import pandas as pd

from .check_types import check_types
from .engine import Job, session_device
from .frames import ExpectationFrame, GammaFrame
from .params import Params

logger = logging.getLogger(__name__)


def _as_gamma_frame(df_with_gamma, params: Params, settings, spark) -> GammaFrame:
    if isinstance(df_with_gamma, GammaFrame):
        return df_with_gamma
    from .blocking import as_pandas
    df = as_pandas(df_with_gamma)
    names = list(params._gamma_cols)
    missing = [n for n in names if n not in df.columns]
    if missing:
        raise ValueError(f"df_with_gamma lacks the gamma columns {missing}")
    levels = [params.params["π"][n]["num_levels"] for n in names]
    gam = df[names].to_numpy(dtype=np.int64)
    job = Job.from_gamma_table(df, names, session_device(spark))
    return GammaFrame(job, settings, program=(names, levels), gammas=gam.astype(np.int8))


@check_types
def run_expectation_step(df_with_gamma: object, params: Params, settings: dict, spark: object, compute_ll=False):
    gf = _as_gamma_frame(df_with_gamma, params, settings, spark)
    if compute_ll:
        ll = get_overall_log_likelihood(gf, params, spark)
        logger.info(f"Log likelihood for iteration {params.iteration - 1}:  {ll}")
        params.params["log_likelihood"] = ll
    return ExpectationFrame(gf, settings, params.params["λ"], params._level_probabilities())


def get_overall_log_likelihood(df_with_gamma_probs, params, spark):
    """Σ ln(λ·Πm + (1-λ)·Πu) over all pairs (expectation_step.py:224-272), via the pattern histogram."""
    gf = df_with_gamma_probs.gammas if isinstance(df_with_gamma_probs, ExpectationFrame) else df_with_gamma_probs
    gf.ensure_codes()
    return gf.job.log_likelihood(params.params["λ"], params._level_probabilities())
