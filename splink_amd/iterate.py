"""EM driver loop (reference: splink/iterate.py:19-65)."""
import logging
from typing import Callable

from .check_types import check_types
from .expectation_step import run_expectation_step
from .maximisation_step import run_maximisation_step
from .params import Params

logger = logging.getLogger(__name__)


@check_types
def iterate(df_gammas: object, params: Params, settings: dict, spark: object, compute_ll: bool = False,
            save_state_fn: Callable = None):
    """Run E and M steps until convergence or max_iterations, then one final E-step."""
    for i in range(settings["max_iterations"]):
        df_e = run_expectation_step(df_gammas, params, settings, spark, compute_ll=compute_ll)
        if not hasattr(df_gammas, "ensure_codes"):
            df_gammas = df_e.gammas  # upload a host gamma table once
        run_maximisation_step(df_e, params, spark)
        logger.info(f"Iteration {i} complete")
        if save_state_fn:
            save_state_fn(params, settings)
        if params.is_converged():
            logger.info("EM algorithm has converged")
            break
    # the returned frame reflects the parameters of the last M-step
    return run_expectation_step(df_gammas, params, settings, spark, compute_ll=compute_ll)
