"""Ordinal windows of spk_gammas and other regressions of the context's bookkeeping (through the C ABI).

The reference joins and projects any number of pairs (blocking.py:95-160, gammas.py:65-89); the device
pass runs a pair set of more than ~2^31 pairs as consecutive ordinal windows (include/splink_hip.h,
spk_gammas_set_window).  Here the window is forced small so that many windows run over a few million
pairs, and every comparison vector must equal the one-window pass and the oracle: windows that split a
blocking rule, the implied-level ranges, the rule-1 view launch, the interpreter path and a link_only job.
The pass over more than 2^31 real pairs is tests/test_gpu_scale.py::test_cfg4_shard_full_size[0of2].
"""
import numpy as np
import pytest

import oracle as orc

pytestmark = pytest.mark.gpu

COLS = ["first_name", "surname", "dob", "city", "email"]
SPECS = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]


@pytest.fixture(scope="module")
def amd():
    from splink_amd import AmdSession, _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    return AmdSession(0)


def _records(n, seed):
    from splink_amd.synthetic import make_records
    return make_records(n, seed=seed, surname_vocab=max(n // 40, 50), first_vocab=300,
                        city_vocab=60)[["unique_id"] + COLS]


@pytest.fixture(scope="module")
def dedupe_job(amd):
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import cfg_settings
    st = complete_settings_dict(cfg_settings(2), amd)
    job = Job("dedupe_only", [_records(60000, 41)], "unique_id", 0)
    job.block(st["blocking_rules"])
    job.gammas(st)
    ref = job.gammas_host()
    table = job.tables[0]
    l, r = job.pair_rows()
    cols = [orc.StrCol(table[c].tolist()) for c in COLS]
    assert (ref == orc.template_gammas(SPECS, cols, cols, l, r)).all()
    return job, st, ref


@pytest.mark.parametrize("size", ["tiny", "odd", "fifth"])
@pytest.mark.parametrize("mode", [1, 21, 0])  # filter, filter + forced rule-1 view launch, interpreter
def test_windows_give_identical_codes(dedupe_job, size, mode):
    job, st, ref = dedupe_job
    P = job.n_pairs
    window = {"tiny": 1000, "odd": 4096 + 17, "fifth": P // 5 + 1}[size]
    assert P > 4 * window  # several windows, and rule 1's pairs start inside one of them
    job.ctx.gammas_set_simple(mode)
    job.ctx.gammas_set_window(0)
    job.gammas(st)
    one = job.gammas_host()
    exact_one = job.ctx.gammas_exact_counts(len(COLS))
    job.ctx.gammas_set_window(window)
    try:
        job.gammas(st)
        got = job.gammas_host()
        n_win = job.ctx.gammas_windows()
        exact = job.ctx.gammas_exact_counts(len(COLS))
        # the E+M launch over codes written window by window
        lam, m, u = 0.2, [], []
        for L in job.code_meta[1]:
            pm = np.linspace(1.0, 3.0, L)
            m += list(pm / pm.sum())
            u += list(pm[::-1] / pm.sum())
        n_stats = 5 + 4 * sum(L + 1 for L in job.code_meta[1])
        stats_w = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
    finally:
        job.ctx.gammas_set_window(0)
        job.ctx.gammas_set_simple(1)
    # windows of equal size, a multiple of 64 pairs, none of them empty (the count follows from that size)
    def cdiv(a, b):
        return -(-a // b)
    w_size = cdiv(cdiv(P, cdiv(P, window)), 64) * 64
    assert n_win == cdiv(P, w_size) and n_win >= 4 and (n_win - 1) * w_size < P
    assert (one == ref).all() and (got == ref).all(), np.nonzero((got != ref).any(axis=1))[0][:10]
    assert exact == exact_one  # the filter decides each cell alone: the same cells reach the exact passes
    job.gammas(st)
    stats_1 = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
    assert np.array_equal(stats_w, stats_1)


def _em_args(job):
    lam, m, u = 0.2, [], []
    for L in job.code_meta[1]:
        pm = np.linspace(1.0, 3.0, L)
        m += list(pm / pm.sum())
        u += list(pm[::-1] / pm.sum())
    return lam, m, u, 5 + 4 * sum(L + 1 for L in job.code_meta[1])


@pytest.mark.parametrize("mode,lev", [(1, 2), (21, 2), (0, 2), (101, 2), (1, 0), (1, 1), (1, 3), (101, 1)])
def test_two_stream_split_gives_identical_codes(dedupe_job, mode, lev):
    """spk_gammas_set_streams: the pair set as two windows at once, the second on a stream of its own (forced
    here at any size).  Codes, exact-pass cell counts and the E+M statistics equal the one-stream pass: the
    filter, the interpreter, forced view launches, every slow-list launch left to the settlement of both windows
    (+100), and every Levenshtein kernel mode."""
    job, st, ref = dedupe_job
    lam, m, u, n_stats = _em_args(job)
    job.ctx.gammas_set_simple(mode)
    job.ctx.gammas_set_lev_kernel(lev)
    try:
        job.ctx.gammas_set_streams(1)
        job.gammas(st)
        one = job.gammas_host()
        exact_one = job.ctx.gammas_exact_counts(len(COLS))
        list_one = np.sort(job.ctx.gammas_exact_list(4, exact_one[4]))
        stats_1 = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
        job.ctx.gammas_set_streams(2, 0)
        job.gammas(st)
        assert job.ctx.gammas_windows() == 2
        # the E+M launch queued right behind the split pass (its codes settled through both windows first)
        stats_2 = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
        got = job.gammas_host()
        exact = job.ctx.gammas_exact_counts(len(COLS))
        list_two = np.sort(job.ctx.gammas_exact_list(4, exact[4]))  # both windows' lists, global ordinals
        # two split passes back to back (the first left pending) and a read after the second
        job.gammas(st)
        job.gammas(st)
        again = job.gammas_host()
    finally:
        job.ctx.gammas_set_streams(2)
        job.ctx.gammas_set_simple(1)
        job.ctx.gammas_set_lev_kernel(2)
    assert (one == ref).all()
    assert (got == ref).all(), np.nonzero((got != ref).any(axis=1))[0][:10]
    assert (again == ref).all()
    assert exact == exact_one
    assert np.array_equal(list_two, list_one)
    assert np.array_equal(stats_2, stats_1)


@pytest.mark.parametrize("streams,mode", [(2, 1), (1, 1), (2, 101), (2, 21)])
def test_graph_replay_gives_identical_codes(dedupe_job, streams, mode):
    """spk_gammas_set_graph: repeated passes with the same program replay a captured HIP graph (the second call
    captures, later ones replay).  Every pass's codes, exact-pass cells and the E+M statistics equal the directly
    enqueued pass -- split or one stream, with every slow-list launch left to the settlement (+100, restored on
    replay), with the forced rule-1 view launch (+20)."""
    job, st, ref = dedupe_job
    lam, m, u, n_stats = _em_args(job)
    job.ctx.gammas_set_simple(mode)
    try:
        job.ctx.gammas_set_streams(streams, 0)
        job.ctx.gammas_set_graph(False)
        job.gammas(st)
        stats_direct = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
        exact_direct = job.ctx.gammas_exact_counts(len(COLS))
        job.ctx.gammas_set_graph(True)
        before = job.ctx.gammas_graph_launches()
        for _ in range(4):
            job.gammas(st)
            stats = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
            assert np.array_equal(stats, stats_direct)
            assert job.ctx.gammas_exact_counts(len(COLS)) == exact_direct
            assert (job.gammas_host() == ref).all()
        assert job.ctx.gammas_graph_launches() - before >= 2  # calls 3 and 4 (call 2 captured)
        # a different program (one column fewer) is enqueued directly, and the first program again is exact
        st2 = dict(st)
        st2["comparison_columns"] = st["comparison_columns"][:4]
        job.gammas(st2)
        assert (job.gammas_host() == ref[:, :4]).all()
        job.gammas(st)
        assert (job.gammas_host() == ref).all()
    finally:
        job.ctx.gammas_set_graph(False)
        job.ctx.gammas_set_streams(2)
        job.ctx.gammas_set_simple(1)


def test_two_stream_split_exact_ms(dedupe_job):
    """The split pass reports an exact launch's time as the sum of its two windows' launches (spk_gammas_exact_ms),
    the one-stream pass as its one launch."""
    job, st, ref = dedupe_job
    job.ctx.enable_timing(True, exact=True)
    try:
        job.ctx.gammas_set_streams(2, 0)
        job.gammas(st)
        ms2 = job.ctx.gammas_exact_ms(len(COLS))
        job.ctx.gammas_set_streams(1)
        job.gammas(st)
        ms1 = job.ctx.gammas_exact_ms(len(COLS))
    finally:
        job.ctx.gammas_set_streams(2)
        job.ctx.enable_timing(False)
    for k in (0, 4):  # the fused JW launch (timed under its first column, first_name), email
        assert ms1[k] > 0 and ms2[k] > 0, (k, ms1, ms2)


def test_windows_link_only(amd):
    """link_only (two tables, asymmetric sides) with three rules, windows of 3000 pairs."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import cfg_settings
    df = _records(30000, 43)
    st = cfg_settings(2)
    st["link_type"] = "link_only"
    st["blocking_rules"] = ["l.surname = r.surname", "l.dob = r.dob", "l.email = r.email"]
    st = complete_settings_dict(st, amd)
    inputs = [df.iloc[:15000].reset_index(drop=True), df.iloc[15000:].reset_index(drop=True)]
    job = Job("link_only", inputs, "unique_id", 0)
    job.block(st["blocking_rules"])
    job.ctx.gammas_set_window(3000)
    try:
        job.gammas(st)
        got = job.gammas_host()
        assert job.ctx.gammas_windows() >= 4
    finally:
        job.ctx.gammas_set_window(0)
    l, r = job.pair_rows()
    tl, tr = job.tables[0], job.r_table()
    ref = orc.template_gammas(SPECS, [orc.StrCol(tl[c].tolist()) for c in COLS],
                              [orc.StrCol(tr[c].tolist()) for c in COLS], l, r)
    assert (got == ref).all()


def test_new_column_after_raw_release(amd):
    """gammas() releases the raw string columns; a later upload (a new comparison column, a
    new blocking pass) must get a fresh raw id, never one a live raw column (uid, numeric or host key)
    still holds.  Re-blocking on the same job and adding a comparison column both stay oracle-exact."""
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import _lev3, cfg_settings
    df = _records(8000, 47)
    df["email2"] = df["email"]
    st = complete_settings_dict(cfg_settings(2), amd)
    job = Job("dedupe_only", [df], "unique_id", 0)
    # a host-keyed rule (lower()) uploads an int64 key column next to the uid and the string columns
    rules = ["lower(l.surname) = lower(r.surname)", "l.dob = r.dob"]
    job.block(rules)
    job.gammas(st)  # releases the raw string columns
    st2 = complete_settings_dict(cfg_settings(2), amd)
    st2["comparison_columns"].append({"col_name": "email2", "num_levels": 3, "case_expression": _lev3("email2")})
    st2 = complete_settings_dict(st2, amd)
    job.gammas(st2)  # a new string column: new raw ids after the released ones
    job.block(rules)  # re-block: the key and uid columns must still be the ones uploaded
    job.gammas(st2)
    got = job.gammas_host()
    table = job.tables[0]
    l, r = job.pair_rows()
    cols = [orc.StrCol(table[c].tolist()) for c in COLS + ["email2"]]
    specs = SPECS + [("lev", 3, [0.3])]
    assert (got == orc.template_gammas(specs, cols, cols, l, r)).all()
    sn = table["surname"].str.lower().to_numpy()
    dob = table["dob"].to_numpy()
    uid = table["unique_id"].to_numpy()
    ok = ((sn[l] == sn[r]) & (table["surname"].notna().to_numpy()[l])) | (dob[l] == dob[r])
    assert ok.all() and (uid[l] < uid[r]).all()


@pytest.mark.parametrize("chunked", [False, True])
def test_prefetched_columns_match_direct_upload(amd, chunked):
    """Job(prefetch=...) uploads comparison-only string columns from a background thread while the uid
    ranks and blocking run; the adopted device columns (spk_raw_utf8_arrow, on_device) must give the same
    encoded table (spk_table_digest) and comparison vectors as the direct upload -- Arrow chunks with sliced
    offsets and validity bitmaps included."""
    import pandas as pd
    import pyarrow as pa
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import cfg_settings
    df = _records(20000, 53)
    for c in COLS:  # Arrow-backed; chunked: several chunks, the later ones sliced (nonzero offset base)
        vals = pa.array(df[c].tolist(), type=pa.large_string())
        parts = [vals.slice(0, 7000), vals.slice(7000, 6000), vals.slice(13000)] if chunked else [vals]
        df[c] = pd.Series(pd.arrays.ArrowExtensionArray(pa.chunked_array(parts)))
    st = complete_settings_dict(cfg_settings(2), amd)
    out = []
    for pre in (None, ["first_name", "email", "city"]):
        job = Job("dedupe_only", [df], "unique_id", 0, prefetch=pre)
        job.block(st["blocking_rules"])
        job.gammas(st)
        out.append((job.ctx.table_digest(0), job.gammas_host(), job.timings.get("prefetch_wait_s")))
    assert out[1][2] is not None  # the prefetched columns were adopted
    assert out[0][0] == out[1][0]
    assert (out[0][1] == out[1][1]).all()


def test_prefetch_of_a_derived_only_column_is_dropped(amd):
    """A column the comparison program reads only through a derived expression (jaro_winkler_sim over
    lower(first_name)) is not prefetched by block_using_rules' choice, and a prefetch the program does not
    adopt is dropped once the program is compiled (nothing left pending, its staging tensors released)."""
    from splink_amd.blocking import _comparison_only_columns
    from splink_amd.engine import Job
    from splink_amd.settings import complete_settings_dict
    from splink_amd.synthetic import cfg_settings
    import pyarrow as pa
    import pandas as pd
    df = _records(5000, 54)
    for c in COLS:
        df[c] = pd.Series(pd.arrays.ArrowExtensionArray(pa.chunked_array([pa.array(df[c].tolist(),
                                                                                   type=pa.large_string())])))
    st = cfg_settings(2)
    cc = [dict(c) for c in st["comparison_columns"]]
    cc[0] = {"custom_name": "fn", "custom_columns_used": ["first_name"], "num_levels": 2,
             "case_expression": "case when first_name_l is null or first_name_r is null then -1 "
                                "when jaro_winkler_sim(lower(first_name_l), lower(first_name_r)) > 0.9 then 1 else 0 end"}
    st = complete_settings_dict(dict(st, comparison_columns=cc), amd)
    assert "first_name" not in _comparison_only_columns(st, st["blocking_rules"], [df])
    job = Job("dedupe_only", [df], "unique_id", 0, prefetch=["first_name", "email"])
    job.block(st["blocking_rules"])
    job.gammas(st)
    assert not job._prefetch
    ref = Job("dedupe_only", [df], "unique_id", 0)
    ref.block(st["blocking_rules"])
    ref.gammas(st)
    assert (job.gammas_host() == ref.gammas_host()).all()
