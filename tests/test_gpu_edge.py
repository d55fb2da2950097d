"""Reference edge cases on the HIP path (through the C ABI), against fixtures generated from the reference.

* the first E-step lists of tests/test_expectation.py:57-66 and tests/test_nulls.py:11;
* m = 5.9e-25 through the 35-digit literal (tests/test_spark.py:130-160);
* the log-likelihood of every E-step of iterate(compute_ll=True) (expectation_step.py:52-57, 224-272);
* manually_apply_fellegi_sunter_weights (splink/__init__.py:111-119), the save_state_fn hook
  (splink/iterate.py:54-55) and load_from_json -> Splink (splink/__init__.py:175-194);
* NULL unique ids in dedupe_only and link_and_dedupe (blocking.py:136, :139).
"""
import copy
import json
import warnings

import numpy as np
import pandas as pd
import pytest

from conftest import load_golden
from test_gpu_parity import check_history, compare_frames, frame, rel_close, run_linker, spark_for

pytestmark = pytest.mark.gpu
warnings.filterwarnings("ignore")

EDGE_PIPELINES = ["first_estep_test1", "first_estep_nulls", "tiny_numbers_estep", "tiny_numbers_em",
                  "null_uid_dedupe", "null_uid_link_and_dedupe", "ll_cfg1"]
LL_CASES = ["first_estep_test1", "first_estep_nulls", "tiny_numbers_estep", "tiny_numbers_em", "ll_test1",
            "ll_nulls", "ll_cfg1"]


@pytest.fixture(scope="module")
def amd():
    from splink_amd import AmdSession, _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    return AmdSession(0)


@pytest.mark.parametrize("case", EDGE_PIPELINES)
def test_edge_pipeline_matches_reference(case, amd):
    g = load_golden("edge_cases")[case]
    linker = run_linker(g, amd)
    df_e = linker.get_scored_comparisons()
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])
    check_history(linker.params, g)
    if "reference_literal_mp" in g:  # the reference tests' own literal lists
        got = sorted(df_e.toPandas()["match_probability"].tolist())
        assert got == pytest.approx(sorted(g["reference_literal_mp"]), abs=1e-8)


@pytest.mark.parametrize("case", LL_CASES)
def test_log_likelihood_every_estep(case, amd):
    """iterate(compute_ll=True): params.params['log_likelihood'] after every E-step, kept in the
    parameter history, equals the reference's get_overall_log_likelihood at 1e-9."""
    from splink_amd import Params, add_gammas, block_using_rules, complete_settings_dict, iterate
    g = load_golden("edge_cases")[case]
    spark = spark_for(g["jaro"], amd)
    settings = complete_settings_dict(copy.deepcopy(g["settings_in"]), spark)
    params = Params(settings, spark)
    df_c = block_using_rules(settings, spark, df=frame(g.get("df")), df_l=frame(g.get("df_l")),
                             df_r=frame(g.get("df_r")))
    df_g = add_gammas(df_c, settings, spark)
    df_e = iterate(df_g, params, settings, spark, compute_ll=True)
    got = [h["log_likelihood"] for h in params.param_history] + [params.params["log_likelihood"]]
    assert len(got) == len(g["log_likelihood"])
    for a, b in zip(got, g["log_likelihood"]):
        assert rel_close(a, b), (a, b)
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])


def test_manually_apply_fellegi_sunter_weights(amd):
    """Scores with the settings' m / u and no EM: the reference's first E-step (test_expectation.py:57-66)."""
    from splink_amd import Splink
    g = load_golden("edge_cases")["first_estep_test1"]
    settings = copy.deepcopy(g["settings_in"])
    settings["max_iterations"] = 7  # ignored: no EM runs
    linker = Splink(settings, spark_for(g["jaro"], amd), df=frame(g["df"]))
    df_e = linker.manually_apply_fellegi_sunter_weights()
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])
    assert linker.params.iteration == 1 and linker.params.param_history == []


def test_save_state_fn_called_every_iteration(amd):
    """iterate.py:54-55: save_state_fn(params, settings) after every M-step, before the convergence test."""
    g = load_golden("test1")
    seen = []

    def save_state(params, settings):
        seen.append((params.iteration, params.params["λ"], settings["max_iterations"]))

    from splink_amd import Splink
    linker = Splink(copy.deepcopy(g["settings_in"]), spark_for(g["jaro"], amd), df=frame(g["df"]),
                    save_state_fn=save_state)
    linker.get_scored_comparisons()
    assert [s[0] for s in seen] == list(range(2, 2 + len(g["iterations"])))
    for (_, lam, mi), it in zip(seen, g["iterations"]):
        assert rel_close(lam, it["lambda"]) and mi == g["settings_in"]["max_iterations"]


def test_load_from_json_resumes(amd, tmp_path):
    """save_model_as_json after one iteration, load_from_json, one more iteration: the reference's
    second-iteration parameters and scores (test_spark.py:211-221, 296-311)."""
    from splink_amd import Splink, load_from_json
    g = load_golden("test1")
    spark = spark_for(g["jaro"], amd)
    settings = copy.deepcopy(g["settings_in"])
    settings["max_iterations"] = 1
    linker = Splink(settings, spark, df=frame(g["df"]))
    linker.get_scored_comparisons()
    assert rel_close(linker.params.params["λ"], g["iterations"][0]["lambda"])
    path = str(tmp_path / "model.json")
    linker.save_model_as_json(path)
    saved = json.load(open(path))
    assert set(saved) == {"current_params", "historical_params", "settings"}
    linker2 = load_from_json(path, spark, df=frame(g["df"]))
    assert linker2.params.params == linker.params.params
    df_e = linker2.get_scored_comparisons()
    it2 = g["iterations"][1]
    assert rel_close(linker2.params.params["λ"], it2["lambda"])
    for gname, d in it2["pi"].items():
        for i, (m, u) in enumerate(zip(d["m"], d["u"])):
            assert rel_close(linker2.params.params["π"][gname]["prob_dist_match"][f"level_{i}"]["probability"], m)
            assert rel_close(linker2.params.params["π"][gname]["prob_dist_non_match"][f"level_{i}"]["probability"], u)
    compare_frames(df_e.toPandas(), g["df_e"], g["df_e_columns"])


def _anagram_job(amd, n=40000):
    """A comparison table whose undecided cells outgrow the exact-pass lists on the first spk_gammas call
    (3 Levenshtein columns x 40k anagram pairs), so the codes are corrected after the call returned."""
    from splink_amd.gammas import _job_from_comparison_table
    from splink_amd.settings import complete_settings_dict
    rng = np.random.Generator(np.random.PCG64(33))
    base = np.array(list("abcdefghij"))
    data = {}
    for c in ("x", "y", "z"):
        data[f"{c}_l"] = ["".join(rng.permutation(base)) for _ in range(n)]
        data[f"{c}_r"] = ["".join(rng.permutation(base)) for _ in range(n)]
    expr = ("case when {c}_l is null or {c}_r is null then -1 when levenshtein({c}_l, {c}_r) <= 5 then 2 "
            "when levenshtein({c}_l, {c}_r) <= 7 then 1 else 0 end")
    st = complete_settings_dict({"link_type": "dedupe_only", "comparison_columns": [
        {"custom_name": c, "custom_columns_used": [c], "num_levels": 3, "case_expression": expr.format(c=c)}
        for c in ("x", "y", "z")]}, amd)
    return _job_from_comparison_table(pd.DataFrame(data), amd), st


def test_async_em_iteration_matches_sync(amd):
    """spk_em_iteration_start / _wait (the bench's software-pipelined loop: comparison pass i queued, then
    the M-step of i - 1, then E+M i) give the statistics of the synchronous spk_em_iteration, including
    on the first call, whose codes are corrected after spk_gammas returned (the iteration is re-enqueued);
    a second start without a wait is refused."""
    from splink_amd.engine import m_step_rows
    from splink_amd.params import Params
    job, st = _anagram_job(amd)
    job.ctx.enable_timing(True, exact=True)
    p_sync, p_async = Params(copy.deepcopy(st), amd), Params(copy.deepcopy(st), amd)
    assert p_sync._level_probabilities() == p_async._level_probabilities()
    job.gammas(st)  # first call: the work lists overflow, the correction happens at the EM's wait
    job.em_start(p_async.params["λ"], p_async._level_probabilities())
    with pytest.raises(RuntimeError, match="not waited for"):
        job.em_start(p_async.params["λ"], p_async._level_probabilities())
    a = job.em_wait()
    s = job.em_stats(p_sync.params["λ"], p_sync._level_probabilities())
    assert np.array_equal(a, s, equal_nan=True), np.nonzero(~((a == s) | (np.isnan(a) & np.isnan(s))))
    names, nlev = job.code_meta
    for p in (p_sync, p_async):
        p._update_params(*m_step_rows(s, names, nlev))
    pending = False
    for _ in range(4):  # pipelined: pass i queued before the M-step of i - 1
        job.gammas(st)
        if pending:
            p_async._update_params(*m_step_rows(job.em_wait(), names, nlev))
        job.em_start(p_async.params["λ"], p_async._level_probabilities())
        pending = True
    p_async._update_params(*m_step_rows(job.em_wait(), names, nlev))
    for _ in range(4):  # plain
        job.gammas(st)
        p_sync._update_params(*m_step_rows(job.em_stats(p_sync.params["λ"], p_sync._level_probabilities()),
                                           names, nlev))
    assert p_async.params["λ"] == p_sync.params["λ"]
    assert p_async._level_probabilities() == p_sync._level_probabilities()
    ms = job.ctx.kernel_ms_done()
    assert ms["gamma"] > 0 and ms["em_hist"] > 0
    # each Levenshtein column's exact-pass launch was timed (spk_gammas_exact_ms, bench.py string_rates)
    xms = job.ctx.gammas_exact_ms(3)
    assert all(x > 0 for x in xms), xms


def test_tf_sums_use_the_scores_not_a_later_em_iteration(amd):
    """tf's per-value Σmp come from the last spk_score's parameters (term_frequencies.py:49-65 averages
    the scored df_e's match_probability), even when an E+M iteration with other parameters ran after the
    score (it rewrites the EM's own per-pattern table)."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records
    df = make_records(20_000, surname_vocab=400)[["unique_id", "first_name", "surname", "dob", "city", "email"]]
    params = Params(cfg_settings(2), amd)
    st = params.settings
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    P = job.n_pairs
    assert P > 100_000
    lp = params._level_probabilities()
    mp = job.score(0.2, lp)
    swapped = [(u, m) for m, u in lp]
    job.em_stats(0.6, swapped)  # other parameters: a different mp per pattern
    rng = np.random.Generator(np.random.PCG64(5))
    ids = rng.integers(0, 50, len(df)).astype(np.int64)  # a value id per table row
    s, c = job.ctx.tf_accumulate(50, ids, ids)
    l, r = job.pair_rows()
    ok = (ids[l] == ids[r]) & ~np.isnan(mp)
    assert ok.sum() > 1000
    want = np.bincount(ids[l][ok], weights=mp[ok], minlength=50)
    assert np.array_equal(c, np.bincount(ids[l][ok], minlength=50))
    assert np.allclose(s, want, rtol=1e-12, atol=0.0)


def test_tf_sums_keep_tiny_match_probabilities(amd):
    """Per-value Σmp (term_frequencies.py:49-65) when every pair scores far below 2^-260 (mp ~ 1e-160): the
    sums keep their relative precision (1e-12 against a host sum), so adj_lambda stays the small positive
    mean the reference computes instead of 0 (parameters as tests/test_spark.py:130-160's tiny m, pushed
    further).  The m values stay >= 1e-33: the E-step's 35-decimal literal (expectation_step.py:212) turns
    anything below 1e-35 into 0."""
    import pandas as pd
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records
    df = make_records(20_000, surname_vocab=400)[["unique_id", "first_name", "surname", "dob", "city", "email"]]
    params = Params(cfg_settings(2), amd)
    st = params.settings
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    tiny = []
    for k, (m, u) in enumerate(params._level_probabilities()):
        tiny.append(([1e-33 * (j + 1) * (k + 1) for j in range(len(m))], list(u)))
    codes, _ = pd.factorize(job.tables[0]["surname"], use_na_sentinel=True)
    codes = codes.astype(np.int64)
    n = int(codes.max()) + 1
    l, r = job.pair_rows()
    for lam in (1e-3, 0.2):
        mp = job.score(lam, tiny)
        # patterns with most columns null keep a single m/u factor (mp up to ~1e-34); the bulk is ~1e-160
        assert np.nanmax(mp) < 1e-30 and np.nanmedian(mp) < 1e-100 and np.nanmin(mp) > 0.0
        s, c = job.ctx.tf_accumulate(n, codes, codes)  # host value ids: the same scale and sum kernels
        ok = (codes[l] >= 0) & (codes[l] == codes[r]) & ~np.isnan(mp)
        want = np.bincount(codes[l][ok], weights=mp[ok], minlength=n)
        assert np.array_equal(c, np.bincount(codes[l][ok], minlength=n))
        has = c > 0
        assert has.sum() > 50 and (s[has] > 0.0).all()
        assert np.allclose(s, want, rtol=1e-12, atol=0.0)


def test_chunked_arrow_ingest_matches_combined(amd):
    """A string column handed over as a multi-chunk Arrow array (spk_raw_utf8_arrow_chunks: no host-side
    combine) encodes to the same device table as the combined column: uneven chunks, sliced chunks (a
    nonzero first offset and validity bit offset), NULLs and empty strings; pairs and comparison vectors
    equal too."""
    import pyarrow as pa
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records
    cols = ["first_name", "surname", "dob", "city", "email"]
    df = make_records(30_000, seed=44, surname_vocab=500, arrow=True)[["unique_id"] + cols].copy()
    df.loc[5, "email"] = ""
    chunked = df.copy()
    cuts = [0, 1, 7, 4000, 4001, 17_333, 30_000]
    for c in ("first_name", "surname", "city", "email"):
        whole = pa.array(df[c].array._pa_array.to_pylist(), type=pa.large_string())
        padded = pa.concat_arrays([pa.array(["x", None, "yz"], type=pa.large_string()), whole])
        parts = [padded.slice(3 + a, b - a) for a, b in zip(cuts[:-1], cuts[1:])]
        chunked[c] = pd.Series(pd.arrays.ArrowExtensionArray(pa.chunked_array(parts)), index=df.index)
    assert chunked["email"].array._pa_array.num_chunks == len(cuts) - 1
    st = Params(cfg_settings(2), amd).settings
    jobs = []
    for frame_ in (df, chunked):
        job = Job("dedupe_only", [frame_], "unique_id", 0)
        job.block(st["blocking_rules"])
        job.gammas(st)
        jobs.append(job)
    a, b = jobs
    assert a.ctx.table_digest(0) == b.ctx.table_digest(0)
    la, ra = a.pair_rows()
    lb, rb = b.pair_rows()
    assert np.array_equal(la, lb) and np.array_equal(ra, rb)
    assert np.array_equal(a.gammas_host(), b.gammas_host())


def test_tf_adjusted_tiny_mp_link_only_matches_oracle(amd):
    """tf adjustment (term_frequencies.py:49-117) on a link_only frame whose match probabilities are all
    tiny: the m probabilities follow the reference's tiny_numbers case (tests/test_spark.py:137-150,
    m = 5.9e-25 for a level) on every column, so mp per pair sits far below 2^-260.  The per-value sums
    keep their relative precision (per-value scale + fixed-point limbs), so every pair's
    tf_adjusted_match_prob equals oracle.tf_adjust_codes over host-factorised surnames at 1e-9; an
    exponent-blind fixed point would give adj_lambda = 0 and a different tf_adjusted_match_prob."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records
    from splink_amd.term_frequencies import _bayes_pair
    import oracle as orc
    df = make_records(40_000, seed=45, surname_vocab=700)[["unique_id", "first_name", "surname", "dob", "city", "email"]]
    a, b = df.iloc[:20_000].reset_index(drop=True), df.iloc[20_000:].reset_index(drop=True)
    settings = cfg_settings(2)
    settings["link_type"] = "link_only"
    for c in settings["comparison_columns"]:
        if c["col_name"] == "surname":
            c["term_frequency_adjustments"] = True
    params = Params(settings, amd)
    st = params.settings
    job = Job("link_only", [a, b], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    tiny = [([5.9380419956766985e-25 * (j + 1) for j in range(len(m))], list(u)) for m, u in params._level_probabilities()]
    lam = 0.4
    mp = job.score(lam, tiny)
    assert np.nanmax(mp) < 1e-20 and np.nanmedian(mp) < 1e-78 and np.nanmin(mp) > 0.0
    col = job._col_index[("surname", "str")]
    n_values = job.ctx.tf_column_values(col)
    sums, counts = job.ctx.tf_accumulate_column(col, n_values)
    with np.errstate(invalid="ignore", divide="ignore"):
        adj_lambda = np.where(counts > 0, sums / np.maximum(counts, 1), np.nan)
    has = counts > 0
    assert has.sum() > 50 and (adj_lambda[has] > 0.0).all()
    table = _bayes_pair(adj_lambda, float(1 - lam))
    tf_mp, _ = job.ctx.tf_apply_columns([col], [table], 0, job.n_pairs, want_adj=False)
    l, r = job.pair_rows()
    vl = job.inputs[0]["surname"] if job.perm[0] is None else job.inputs[0]["surname"].take(np.asarray(job.perm[0])).reset_index(drop=True)
    vr = job.inputs[1]["surname"] if job.perm[1] is None else job.inputs[1]["surname"].take(np.asarray(job.perm[1])).reset_index(drop=True)
    codes, _ = pd.factorize(pd.concat([vl, vr], ignore_index=True), use_na_sentinel=True)
    want, _ = orc.tf_adjust_codes(codes[:len(vl)][l], codes[len(vl):][r], mp, lam)
    assert np.allclose(tf_mp, want, rtol=1e-9, atol=0, equal_nan=True)


def test_tf_results_kept_on_device(amd):
    """spk_tf_apply_columns with out_tf_mp = NULL keeps tf_adjusted_match_prob on the device (as spk_score keeps mp);
    spk_tf_copy reads ranges of it back, bit-identical to the host-copy form; ranges outside the applied pairs and a
    replaced pair set are refused (term_frequencies.py:159-168)."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records
    from splink_amd.term_frequencies import _bayes_pair
    df = make_records(30_000, seed=46, surname_vocab=600)[["unique_id", "first_name", "surname", "dob", "city", "email"]]
    a, b = df.iloc[:15_000].reset_index(drop=True), df.iloc[15_000:].reset_index(drop=True)
    settings = cfg_settings(2)
    settings["link_type"] = "link_only"
    params = Params(settings, amd)
    st = params.settings
    job = Job("link_only", [a, b], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    lam = 0.3
    job.score(lam, params._level_probabilities(), want_host=False)
    col = job._col_index[("surname", "str")]
    n_values = job.ctx.tf_column_values(col)
    sums, counts = job.ctx.tf_accumulate_column(col, n_values)
    with np.errstate(invalid="ignore", divide="ignore"):
        adj_lambda = np.where(counts > 0, sums / np.maximum(counts, 1), np.nan)
    table = _bayes_pair(adj_lambda, float(1 - lam))
    P = job.n_pairs
    assert P > 10_000
    host, _ = job.ctx.tf_apply_columns([col], [table], 0, P, want_adj=False)
    with pytest.raises(RuntimeError):  # the host form keeps nothing on the device
        job.ctx.tf_copy(0, 1)
    assert job.ctx.tf_apply_columns([col], [table], 0, P, want_adj=False, want_host=False)[0] is None
    assert np.array_equal(job.ctx.tf_copy(0, P), host, equal_nan=True)
    s0, n = P // 3, P // 4
    assert np.array_equal(job.ctx.tf_copy(s0, n), host[s0:s0 + n], equal_nan=True)
    job.ctx.tf_apply_columns([col], [table], s0, n, want_adj=False, want_host=False)  # a range of the pairs
    assert np.array_equal(job.ctx.tf_copy(s0 + 5, 100), host[s0 + 5:s0 + 105], equal_nan=True)
    with pytest.raises(ValueError):
        job.ctx.tf_copy(0, 10)
    with pytest.raises(ValueError):
        job.ctx.tf_copy(s0 + n - 5, 10)
    assert job.ctx.memory()["em_score_tf"] >= n * 8
    job.block(st["blocking_rules"])  # a new pair set: the kept results no longer describe it
    with pytest.raises(RuntimeError):
        job.ctx.tf_copy(0, 1)


@pytest.mark.parametrize("link_type", ["dedupe_only", "link_only"])
def test_tf_histogram_matches_sort(amd, link_type):
    """The tf sums from the direct (value, pattern) histogram (spk_tf_set_mode 0, the default when n_values x
    n_patterns fits) equal the keys + radix sort + run-length encode form (mode 1: 32-bit keys; mode 2: 64-bit) exactly: scales, fixed-point limbs,
    counts, and tf_adjusted_match_prob (term_frequencies.py:49-65, :122-168); through the device-id and the host-id
    entry points, and with the scale pass's counts reused by the sum pass."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records
    from splink_amd import table as T
    from splink_amd.term_frequencies import _bayes_pair
    df = make_records(30_000, seed=47, surname_vocab=500)[["unique_id", "first_name", "surname", "dob", "city", "email"]]
    settings = cfg_settings(2)
    settings["link_type"] = link_type
    params = Params(settings, amd)
    st = params.settings
    if link_type == "link_only":
        job = Job("link_only", [df.iloc[:15_000].reset_index(drop=True), df.iloc[15_000:].reset_index(drop=True)],
                  "unique_id", 0)
    else:
        job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    lam = 0.2
    job.score(lam, params._level_probabilities(), want_host=False)
    col = job._col_index[("surname", "str")]
    n_values = job.ctx.tf_column_values(col)
    got = {}
    for mode in (0, 1, 2):
        job.ctx.tf_set_mode(mode)
        scale = job.ctx.tf_scales_column(col, n_values)
        limbs, counts = job.ctx.tf_accumulate_column_exact(col, n_values, scale)
        sums, counts2 = job.ctx.tf_accumulate_column(col, n_values)
        with np.errstate(invalid="ignore", divide="ignore"):
            table = _bayes_pair(np.where(counts2 > 0, sums / np.maximum(counts2, 1), np.nan), float(1 - lam))
        tf_mp, _ = job.ctx.tf_apply_columns([col], [table], 0, job.n_pairs, want_adj=False)
        sides = (0, 1) if link_type == "link_only" else (0,)  # host value ids (the non-device-id entry points)
        vals = [pd.Series([None if T.is_null_scalar(v) else v for v in job.host_values(s, "surname").tolist()],
                          dtype=object) for s in sides]
        codes, nv = T.factorize_joint(vals)
        ids0, ids1 = codes[0], (codes[1] if len(codes) > 1 else codes[0])
        scale_h = job.ctx.tf_scales(nv, ids0, ids1)
        limbs_h, counts_h = job.ctx.tf_accumulate_exact(nv, ids0, ids1, scale_h)
        got[mode] = (scale, limbs, counts, sums, counts2, tf_mp, scale_h, limbs_h, counts_h)
    job.ctx.tf_set_mode(0)
    assert (got[0][2] > 0).sum() > 50
    for mode in (1, 2):
        for a, b in zip(got[0], got[mode]):
            assert np.array_equal(a, b, equal_nan=True)
