"""splink_amd: splink's pairwise-comparison + EM hot path on AMD Instinct MI355X (gfx950).

Drop-in for the reference's public API (splink 0.1.7, splink/__init__.py):

    from splink_amd import Splink, load_from_json, AmdSession
    linker = Splink(settings, AmdSession(), df=records)      # pandas / pyarrow / Spark input
    df_e = linker.get_scored_comparisons()                   # device-resident frame
    df_e.toPandas()

Blocking, comparison vectors, EM and scoring run as hand-written HIP kernels in
libsplink_hip.so (C ABI: include/splink_hip.h); there is no CPU fallback.
"""
from typing import Callable

from .blocking import block_using_rules
from .case_statements import _check_jaro_registered
from .check_types import check_types
from .expectation_step import run_expectation_step
from .frames import SplinkDataFrame
from .gammas import add_gammas
from .iterate import iterate
from .params import Params, load_params_from_json
from .session import AmdSession, session
from .settings import complete_settings_dict
from .term_frequencies import make_adjustment_for_term_frequencies
from .validate import validate_settings

__all__ = ["Splink", "load_from_json", "AmdSession", "session", "Params", "block_using_rules", "add_gammas",
           "iterate", "run_expectation_step", "make_adjustment_for_term_frequencies", "complete_settings_dict"]


def _is_frame(x):
    return x is not None and (hasattr(x, "toPandas") or hasattr(x, "to_pandas") or hasattr(x, "columns"))


class Splink:
    """splink data linker (reference splink/__init__.py:33-172)."""

    @check_types
    def __init__(self, settings: dict, spark: object, df_l: object = None, df_r: object = None, df: object = None,
                 save_state_fn: Callable = None):
        self.spark = spark
        _check_jaro_registered(spark)
        settings = complete_settings_dict(settings, spark)
        validate_settings(settings)
        self.settings = settings
        self.params = Params(settings, spark)
        self.df_r = df_r
        self.df_l = df_l
        self.df = df
        self.save_state_fn = save_state_fn
        self._check_args()

    def _check_args(self):
        link_type = self.settings["link_type"]
        if link_type == "dedupe_only":
            if not (self.df_r is None and self.df_l is None and _is_frame(self.df)):
                raise ValueError(
                    "For link_type = 'dedupe_only', you must pass a single Spark dataframe to Splink using the df "
                    "argument. The df_l and df_r arguments should be omitted or set to None. "
                    "e.g. linker = Splink(settings, spark, df=my_df)")
        if link_type in ("link_only", "link_and_dedupe"):
            if not (_is_frame(self.df_l) and _is_frame(self.df_r) and self.df is None):
                raise ValueError(
                    f"For link_type = '{link_type}', you must pass two Spark dataframes to Splink using the df_l and "
                    "df_r argument. The df argument should be omitted or set to None. "
                    "e.g. linker = Splink(settings, spark, df_l=my_first_df, df_r=df_to_link_to_first_one)")

    def _get_df_comparison(self):
        if self.settings["link_type"] == "dedupe_only":
            return block_using_rules(self.settings, self.spark, df=self.df)
        return block_using_rules(self.settings, self.spark, df_l=self.df_l, df_r=self.df_r)

    def manually_apply_fellegi_sunter_weights(self):
        """Match probabilities from the m / u in the settings (no EM)."""
        df_gammas = add_gammas(self._get_df_comparison(), self.settings, self.spark)
        return run_expectation_step(df_gammas, self.params, self.settings, self.spark)

    def get_scored_comparisons(self):
        """Estimate the parameters with EM and return scored comparisons (no tf adjustment)."""
        df_gammas = add_gammas(self._get_df_comparison(), self.settings, self.spark)
        df_gammas.persist()
        df_e = iterate(df_gammas, self.params, self.settings, self.spark, compute_ll=False,
                       save_state_fn=self.save_state_fn)
        df_gammas.unpersist()
        return df_e

    def make_term_frequency_adjustments(self, df_e: SplinkDataFrame):
        return make_adjustment_for_term_frequencies(df_e, self.params, self.settings, retain_adjustment_columns=True,
                                                    spark=self.spark)

    def save_model_as_json(self, path: str, overwrite=False):
        self.params.save_params_to_json_file(path, overwrite=overwrite)


def load_from_json(path: str, spark=None, df_l=None, df_r=None, df=None, save_state_fn: Callable = None):
    """Re-create a linker from save_model_as_json output (reference __init__.py:175-194)."""
    params = load_params_from_json(path)
    linker = Splink(params.settings, spark, df_l, df_r, df, save_state_fn)
    linker.params = params
    return linker
