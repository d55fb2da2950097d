"""Candidate-pair generation (reference: splink/blocking.py:162-318).

`block_using_rules` keeps the reference's signature and semantics: one equi-join per rule,
each excluding pairs an earlier rule produced, the link-type predicate (`l.uid < r.uid` for
dedupe_only, source-table ordering for link_and_dedupe), and a cartesian product when there
are no rules.  The pairs are generated on the GPU (spk_block) and stay there.
"""
import pandas as pd

from .check_types import check_types
from .engine import Job, columns_to_retain_blocking, distributed_shard, session_device, string_columns_read
from .frames import ComparisonFrame


def as_pandas(df):
    """Input tables: pandas, pyarrow Table, or anything with toPandas() (e.g. a Spark DataFrame)."""
    if df is None or isinstance(df, pd.DataFrame):
        return df
    if hasattr(df, "toPandas"):
        return df.toPandas()
    if hasattr(df, "to_pandas"):
        return df.to_pandas()
    raise TypeError(f"unsupported input table type {type(df)}")


def _vertically_concatenate_datasets(df_l, df_r, settings, spark=None):
    """link_and_dedupe: retained columns of both inputs with _source_table 'left' / 'right' (:70-93)."""
    cols = columns_to_retain_blocking(settings)
    left = as_pandas(df_l)[cols].assign(_source_table="left")
    right = as_pandas(df_r)[cols].assign(_source_table="right")
    return pd.concat([left, right], ignore_index=True)


def _tables(settings, df_l, df_r, df):
    lt = settings["link_type"]
    if lt == "dedupe_only":
        return [as_pandas(df)]
    if lt == "link_only":
        return [as_pandas(df_l), as_pandas(df_r)]
    return [_vertically_concatenate_datasets(df_l, df_r, settings)]


def _block(settings, spark, df_l, df_r, df, rules):
    tables = _tables(settings, df_l, df_r, df)
    # comparison-only string columns start their upload at once, behind the unique-id ranks and the blocking
    # work (Job.prefetch_strings)
    job = Job(settings["link_type"], tables, settings["unique_id_column_name"], session_device(spark),
              shard=distributed_shard(), prefetch=_comparison_only_columns(settings, rules, tables))
    job.block(list(rules))
    return ComparisonFrame(job, settings)


def _comparison_only_columns(settings, rules, tables):
    """Input string columns the comparison program reads as bare operands that no blocking rule mentions
    (those are uploaded by the blocking pass itself, which must not wait behind a prefetch).  A column read
    only through a derived expression (`lower(first_name_l)`) is not one: the derived column is what goes to
    the device."""
    import re
    used = set(re.findall(r"[a-z_][a-z_0-9]*", " ".join(rules).lower()))
    try:
        names = string_columns_read(settings, tables)
    except Exception:  # noqa: BLE001 -- only a prefetch: the program's own error surfaces in add_gammas
        return []
    return [c for c in names if c.lower() not in used]


@check_types
def block_using_rules(settings: dict, spark: object, df_l: object = None, df_r: object = None, df: object = None):
    """Candidate pairs for the settings' blocking rules; cartesian product if there are none."""
    if "blocking_rules" not in settings or len(settings["blocking_rules"]) == 0:
        return cartesian_block(settings, spark, df_l, df_r, df)
    return _block(settings, spark, df_l, df_r, df, settings["blocking_rules"])


def cartesian_block(settings: dict, spark, df_l=None, df_r=None, df=None):
    """All pairs allowed by the link type (blocking.py:271-318)."""
    return _block(settings, spark, df_l, df_r, df, [])
