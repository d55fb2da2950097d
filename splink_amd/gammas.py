"""Comparison vectors (reference: splink/gammas.py:92-124).

`add_gammas` evaluates every comparison column's CASE expression over the candidate pairs on
the GPU (spk_gammas) and returns a frame whose `toPandas()` has the reference's columns
(gammas.py:25-62).  It also accepts a pandas comparison table with `<col>_l` / `<col>_r`
columns, as the reference's SQL does.
"""
import numpy as np
import pandas as pd

from .check_types import check_types
from .engine import Job, session_device
from .frames import ComparisonFrame, GammaFrame
from .settings import complete_settings_dict


def _job_from_comparison_table(df: pd.DataFrame, spark):
    left = {c[:-2]: df[c] for c in df.columns if c.endswith("_l")}
    right = {c[:-2]: df[c] for c in df.columns if c.endswith("_r")}
    tl, tr = pd.DataFrame(left), pd.DataFrame(right)
    job = Job("link_only", [tl, tr], "", session_device(spark))
    idx = np.arange(len(df), dtype=np.int32)
    job.load_pairs(idx, idx)
    return job


@check_types
def add_gammas(df_comparison: object, settings_dict: dict, spark: object, unique_id_col: str = "unique_id"):
    settings_dict = complete_settings_dict(settings_dict, spark)
    if isinstance(df_comparison, ComparisonFrame):
        job = df_comparison.job
    else:
        from .blocking import as_pandas
        job = _job_from_comparison_table(as_pandas(df_comparison), spark)
    return GammaFrame(job, settings_dict)
