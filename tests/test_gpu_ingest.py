"""Device ingest (spk_raw_* / spk_key_build / spk_rank_from_raw / spk_cluster / spk_table_add_raw_utf8)
against the oracle's sqlite restatement of blocking.py:95-160.

Blocking keys are hashed, sorted and densified on the GPU from the columns' Arrow buffers; these
tests replay rule shapes the reference accepts -- plain, multi-term, substr (code points), numeric,
asymmetric (`l.a = r.b`), lower() (host-keyed term) -- with NULLs and non-ASCII values, for
dedupe_only, link_only and link_and_dedupe, from pandas object columns and from Arrow-backed columns.
"""
import copy
import warnings

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

import oracle as orc
from conftest import load_golden
from test_gpu_parity import check_history, compare_frames, frame, spark_for

pytestmark = pytest.mark.gpu
warnings.filterwarnings("ignore")


@pytest.fixture(scope="module")
def amd():
    from splink_amd import AmdSession, _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    return AmdSession(0)


def _records(n, seed):
    from splink_amd.synthetic import make_records
    df = make_records(n, seed=seed, surname_vocab=60, first_vocab=50, city_vocab=12)
    df = df[["unique_id", "first_name", "surname", "dob", "city"]].copy()
    rng = np.random.Generator(np.random.PCG64(seed))
    df["age"] = rng.integers(18, 30, len(df)).astype(float)
    df.loc[rng.random(len(df)) < 0.1, "age"] = np.nan
    df["n_kids"] = rng.integers(0, 4, len(df)).astype(np.int64)
    return df


RULES = [
    ["l.surname = r.surname"],
    ["l.first_name = r.first_name AND l.city = r.city", "l.dob = r.dob"],
    ["substr(l.surname, 1, 3) = substr(r.surname, 1, 3)"],
    ["substr(l.dob, 1, 7) = substr(r.dob, 1, 7) AND l.n_kids = r.n_kids"],
    ["l.age = r.age", "l.city = r.city"],
    ["l.first_name = r.surname"],
    ["lower(l.surname) = lower(r.surname)", "substr(l.first_name, 2, 2) = substr(r.first_name, 2, 2)"],
]


def _pair_set(df_c, link_type):
    keys = ["unique_id_l", "unique_id_r"] + (["_source_table_l", "_source_table_r"] if link_type == "link_and_dedupe"
                                             else [])
    return sorted(map(tuple, df_c[keys].astype(str).to_numpy().tolist()))


def _oracle_pair_set(settings, link_type, **dfs):
    pairs, left, right = orc.block(settings, **dfs)
    cmp_df = orc.comparison_frame(pairs, left, right)
    return _pair_set(cmp_df, link_type)


def _arrow(df):
    out = df.copy()
    for c in out.columns:
        if out[c].dtype == object:
            out[c] = pd.Series(pa.array(out[c].tolist(), type=pa.large_string()), dtype=pd.ArrowDtype(pa.large_string()))
    return out


@pytest.mark.parametrize("rules", RULES, ids=[" | ".join(r) for r in RULES])
@pytest.mark.parametrize("link_type", ["dedupe_only", "link_only", "link_and_dedupe"])
def test_device_keys_match_oracle_blocking(amd, rules, link_type):
    from splink_amd.blocking import block_using_rules
    from splink_amd.settings import complete_settings_dict
    df = _records(700, seed=31)
    st = complete_settings_dict({"link_type": link_type, "blocking_rules": rules,
                                 "comparison_columns": [{"col_name": "first_name"}, {"col_name": "surname"},
                                                        {"col_name": "dob"}, {"col_name": "city"},
                                                        {"col_name": "age", "data_type": "numeric"},
                                                        {"col_name": "n_kids", "data_type": "numeric"}]},
                                "supress_warnings")
    if link_type == "dedupe_only":
        dfs = {"df": df}
    else:
        dfs = {"df_l": df.iloc[:350].reset_index(drop=True), "df_r": df.iloc[350:].reset_index(drop=True)}
    want = _oracle_pair_set(st, link_type, **dfs)
    got = _pair_set(block_using_rules(st, amd, **dfs).toPandas(), link_type)
    assert got == want
    # Arrow-backed string columns take the zero-copy path to the same pairs
    got_arrow = _pair_set(block_using_rules(st, amd, **{k: _arrow(v) for k, v in dfs.items()}).toPandas(), link_type)
    assert got_arrow == want


@pytest.mark.parametrize("name", ["test1", "synthetic_cfg1", "custom_exprs", "link_tf"])
def test_arrow_backed_inputs_match_reference(name, amd):
    """The golden pipelines from Arrow-backed string columns (pd.ArrowDtype(large_string)): same pairs,
    comparison vectors, EM and scores as from object columns."""
    from splink_amd import Splink
    g = load_golden(name)
    conv = lambda d: _arrow(frame(d)) if d else None  # noqa: E731
    linker = Splink(copy.deepcopy(g["settings_in"]), spark_for(g["jaro"], amd), df=conv(g.get("df")),
                    df_l=conv(g.get("df_l")), df_r=conv(g.get("df_r")))
    df_e = linker.get_scored_comparisons()
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])
    check_history(linker.params, g)


def test_cluster_permutation_is_consistent(amd):
    """Pair rows index the clustered tables; the host views follow the device permutation."""
    from splink_amd.engine import Job
    df = _records(2000, seed=5)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(["l.surname = r.surname", "l.dob = r.dob"])
    perm = job.perm[0]
    assert sorted(perm.tolist()) == list(range(len(df)))
    view = job.tables[0]
    assert (view["unique_id"].to_numpy() == df["unique_id"].to_numpy()[perm]).all()
    # clustered by the first rule's key: equal surnames are contiguous, NULLs last
    s = view["surname"].tolist()
    seen, prev = set(), object()
    for v in s:
        if v is None:
            continue
        if v != prev:
            assert v not in seen
            seen.add(v)
        prev = v
    nn = view["surname"].isna().to_numpy()
    assert not nn[:len(nn) - nn.sum()].any()
