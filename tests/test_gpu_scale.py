"""Parity at the configs' own sizes (the bench workloads), against the C oracle.

* cfg2 (BASELINE configs[1]): 1M synthetic person records, blocking surname|dob -> 45,981,122 pairs.
  Every comparison vector bit-exact against oracle.template_gammas, 10 EM iterations of λ / m / u and
  the final match_probability at 1e-9 against oracle.em_iterate (case_statements.py:81-141,
  expectation_step.py:167-185, maximisation_step.py:16-90).
* cfg5's columns at 1M records: + the free-text address column (Levenshtein-4, 30-128 characters).
* The pair set at full size through size-independent properties: every pair satisfies a rule and
  the link predicate, no pair repeats, and the count equals the inclusion-exclusion count of the
  two equi-joins computed from the key histograms.
"""
import numpy as np
import pandas as pd
import pytest

import oracle as orc
from test_gpu_parity import rel_close

pytestmark = pytest.mark.gpu

COLS = ["first_name", "surname", "dob", "city", "email"]
SPECS = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3]),
         ("lev", 4, [0.2, 0.4])]
N_RECORDS = 1_000_000
CFG2_PAIRS = 45_981_122  # bench.py's headline workload (BENCH_r01.json config.candidate_pairs)


@pytest.fixture(scope="module")
def amd():
    from splink_amd import AmdSession, _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    return AmdSession(0)


def _c2(n):
    n = n.astype(np.int64)
    return int((n * (n - 1) // 2).sum())


def expected_pair_count(table):
    """|surname join ∪ dob join| for dedupe with unique ids: Σ C(n_s, 2) + Σ C(n_d, 2) - Σ C(n_sd, 2)."""
    s = table["surname"].dropna()
    d = table["dob"].dropna()
    both = table.dropna(subset=["surname", "dob"])
    return (_c2(s.value_counts().to_numpy()) + _c2(d.value_counts().to_numpy())
            - _c2(both.groupby(["surname", "dob"]).size().to_numpy()))


def check_pair_properties(table, l, r):
    uid = table["unique_id"].to_numpy()
    assert (uid[l] < uid[r]).all()
    sn, _ = pd.factorize(table["surname"])  # -1 = NULL
    dob, _ = pd.factorize(table["dob"])
    same_s = (sn[l] >= 0) & (sn[l] == sn[r])
    same_d = (dob[l] >= 0) & (dob[l] == dob[r])
    assert (same_s | same_d).all()
    # rule order: surname pairs first, then dob pairs that are not surname pairs
    n_s = int(same_s.sum())
    assert same_s[:n_s].all() and not same_s[n_s:].any()
    key = l.astype(np.int64) * len(table) + r.astype(np.int64)
    assert len(np.unique(key)) == len(key)
    assert len(key) == expected_pair_count(table)


def run_full(amd, with_address, iters):
    from splink_amd.engine import Job, m_step_rows
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records
    cols = COLS + (["address"] if with_address else [])
    df = make_records(N_RECORDS, surname_vocab=15000, with_address=with_address)[["unique_id"] + cols]
    params = Params(cfg_settings(5 if with_address else 2, max_iterations=iters), amd)
    st = params.settings
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(st["blocking_rules"])
    table = job.tables[0]
    l, r = job.pair_rows()
    check_pair_properties(table, l, r)
    job.gammas(st)
    gam = job.gammas_host()
    ocols = [orc.StrCol(table[c].tolist()) for c in cols]
    ref = orc.template_gammas(SPECS[:len(cols)], ocols, ocols, l, r)
    bad = np.nonzero((gam != ref).any(axis=1))[0]
    assert len(bad) == 0, (len(bad), bad[:5], gam[bad[:5]], ref[bad[:5]])
    del ref, ocols
    names, nlev = job.code_meta
    lam0, lp0 = params.params["λ"], params._level_probabilities()
    hist_o, mp_o = orc.em_iterate(gam, nlev, lam0, [m for m, _ in lp0], [u for _, u in lp0], iters, 1e-300)
    assert len(hist_o) == iters
    for lam_o, m_o, u_o in hist_o:
        stats = job.em_stats(params.params["λ"], params._level_probabilities())
        new_lambda, rows = m_step_rows(stats, names, nlev)
        params._update_params(new_lambda, rows)
        assert rel_close(params.params["λ"], lam_o)
        for k, (m, u) in enumerate(params._level_probabilities()):
            assert all(rel_close(a, b) for a, b in zip(m, m_o[k])), (k, m, m_o[k])
            assert all(rel_close(a, b) for a, b in zip(u, u_o[k])), (k, u, u_o[k])
    mp = job.score(params.params["λ"], params._level_probabilities())
    assert np.allclose(mp, mp_o, rtol=1e-9, atol=0, equal_nan=True)
    return job


def test_cfg2_full_size(amd):
    job = run_full(amd, with_address=False, iters=10)
    assert job.n_pairs == CFG2_PAIRS


def test_cfg5_columns_full_size(amd):
    job = run_full(amd, with_address=True, iters=3)
    assert job.n_pairs > 40_000_000


def rows_of(job, side, rows):
    """Table rows (device row order) of one side as a frame, without materialising the permuted table."""
    perm = job.perm[side]
    return job.inputs[side].take(rows if perm is None else np.asarray(perm)[rows]).reset_index(drop=True)


def column_in_row_order(job, side, col):
    perm = job.perm[side]
    v = job.inputs[side][col]
    return v if perm is None else v.take(np.asarray(perm)).reset_index(drop=True)


def oracle_sample(job, specs, cols, sl, sr):
    """oracle.template_gammas of the pairs (sl[i], sr[i]) (device row order), from only the rows they use."""
    if job.link_type == "link_only":  # rows index the two tables
        ul, il = np.unique(sl, return_inverse=True)
        ur, ir = np.unique(sr, return_inverse=True)
        tl, tr = rows_of(job, 0, ul), rows_of(job, job.r_side(), ur)
        ocl = [orc.StrCol(tl[c].tolist()) for c in cols]
        ocr = [orc.StrCol(tr[c].tolist()) for c in cols]
        return orc.template_gammas(specs, ocl, ocr, il.astype(np.int32), ir.astype(np.int32))
    rows, inv = np.unique(np.concatenate([sl, sr]), return_inverse=True)
    sub = rows_of(job, 0, rows)
    ocols = [orc.StrCol(sub[c].tolist()) for c in cols]
    return orc.template_gammas(specs, ocols, ocols, inv[:len(sl)].astype(np.int32), inv[len(sl):].astype(np.int32))


def check_shard(job, params, cols, iters, sample=2_000_000):
    """Parity of one GPU's share of a big job: every comparison vector of a strided sample of `sample`
    pairs bit-exact against oracle.template_gammas, `iters` EM iterations of λ / m / u and every pair's
    match_probability at 1e-9 against oracle.em_iterate.  Returns (match probabilities, pair rows)."""
    from splink_amd.engine import m_step_rows
    specs = SPECS[:len(cols)]
    l, r = job.pair_rows()
    step = max(1, job.n_pairs // sample)
    idx = np.arange(0, job.n_pairs, step)
    ref = oracle_sample(job, specs, cols, l[idx], r[idx])
    gam = job.gammas_host()
    bad = np.nonzero((gam[idx] != ref).any(axis=1))[0]
    assert len(bad) == 0, (len(bad), idx[bad[:5]])
    del ref
    names, nlev = job.code_meta
    lam0, lp0 = params.params["λ"], params._level_probabilities()
    hist_o, mp_o = orc.em_iterate(gam, nlev, lam0, [m for m, _ in lp0], [u for _, u in lp0], iters, 1e-300)
    del gam
    assert len(hist_o) == iters
    for lam_o, m_o, u_o in hist_o:
        stats = job.em_stats(params.params["λ"], params._level_probabilities())
        new_lambda, rows_ = m_step_rows(stats, names, nlev)
        params._update_params(new_lambda, rows_)
        assert rel_close(params.params["λ"], lam_o)
        for k, (m, u) in enumerate(params._level_probabilities()):
            assert all(rel_close(a, b) for a, b in zip(m, m_o[k])), (k, m, m_o[k])
            assert all(rel_close(a, b) for a, b in zip(u, u_o[k])), (k, u, u_o[k])
    mp = job.score(params.params["λ"], params._level_probabilities())
    assert np.allclose(mp, mp_o, rtol=1e-9, atol=0, equal_nan=True)
    return mp, l, r


def check_shard_streamed(job, params, cols, iters, sample=2_000_000, chunk=1 << 27):
    """check_shard for a pair set too large to hold on the host a few times over (more than 2^31 pairs):
    the comparison vectors are read back chunk by chunk.  A strided sample of `sample` pairs is bit-exact
    against oracle.template_gammas; the oracle's pattern histogram of every pair's comparison vector
    (oracle.pattern_codes: the γ columns as the device decodes them, counted on the host) drives
    `iters` EM iterations of oracle.em_iterate_hist, checked against the device at 1e-9 after every
    M-step; every pair's match_probability is checked against the oracle's mp of its comparison vector."""
    from splink_amd.engine import m_step_rows
    specs = SPECS[:len(cols)]
    names, nlev = job.code_meta
    K, P = len(names), job.n_pairs
    step = max(1, P // sample)
    hist = np.zeros(int(np.prod([L + 1 for L in nlev])), dtype=np.int64)
    sl, sr, sg = [], [], []
    for c0 in range(0, P, chunk):
        n = min(chunk, P - c0)
        g = job.ctx.gammas_copy(K, c0, n)
        orc.pattern_codes(g, nlev, hist, want_codes=False)
        loc = np.arange((-c0) % step, n, step)  # global ordinals k * step
        l, r = job.ctx.pairs_copy(c0, n)
        sl.append(l[loc])
        sr.append(r[loc])
        sg.append(g[loc])
        del g, l, r
    assert int(hist.sum()) == P
    sl, sr, sg = np.concatenate(sl), np.concatenate(sr), np.concatenate(sg)
    assert len(sl) == (P + step - 1) // step
    ref = oracle_sample(job, specs, cols, sl, sr)
    bad = np.nonzero((sg != ref).any(axis=1))[0]
    assert len(bad) == 0, (len(bad), bad[:5] * step)
    lam0, lp0 = params.params["λ"], params._level_probabilities()
    hist_o, mpat_o = orc.em_iterate_hist(hist, nlev, lam0, [m for m, _ in lp0], [u for _, u in lp0], iters, 1e-300)
    assert len(hist_o) == iters
    for lam_o, m_o, u_o in hist_o:
        stats = job.em_stats(params.params["λ"], params._level_probabilities())
        new_lambda, rows_ = m_step_rows(stats, names, nlev)
        params._update_params(new_lambda, rows_)
        assert rel_close(params.params["λ"], lam_o)
        for k, (m, u) in enumerate(params._level_probabilities()):
            assert all(rel_close(a, b) for a, b in zip(m, m_o[k])), (k, m, m_o[k])
            assert all(rel_close(a, b) for a, b in zip(u, u_o[k])), (k, u, u_o[k])
    lam = params.params["λ"]
    m_t, u_t = job.flat_tables(params._level_probabilities())
    for c0 in range(0, P, chunk):
        n = min(chunk, P - c0)
        mp = job.ctx.score(float(lam), float(1 - lam), m_t, u_t, c0, n)
        want = mpat_o[orc.pattern_codes(job.ctx.gammas_copy(K, c0, n), nlev)]
        assert np.allclose(mp, want, rtol=1e-9, atol=0, equal_nan=True), c0


@pytest.fixture(scope="module")
def cfg4_records():
    from splink_amd.synthetic import make_records
    return make_records(20_000_000, surname_vocab=300_000, arrow=True)[["unique_id"] + COLS]


@pytest.mark.parametrize("shard", [(0, 8), (0, 2)], ids=["0of8", "0of2"])
def test_cfg4_shard_full_size(amd, heartbeat, cfg4_records, shard):
    """BASELINE configs[3] at one GPU's share: a 20M-record dedupe (blocking surname | dob: 6.2e9 candidate
    ordinals, past 2^31) whose ordinal space is split over 8 (or 2) GPUs; this process is rank 0 and
    generates only its slice, as each rank of the multi-GPU job does (blocking.py:95-160, int64 ordinals).
    0of8: ~770M pairs; a strided sample of 2M comparison vectors is bit-exact against
    oracle.template_gammas, and 10 EM iterations of λ / m / u plus every pair's match_probability agree
    with oracle.em_iterate at 1e-9.  0of2: ~3.1e9 pairs in ONE context (the 2-GPU split of BASELINE's
    "2/4/8 GPUs"), past 2^31, so the comparison pass runs as ordinal windows (spk_gammas_windows >= 2);
    checked by check_shard_streamed (the same sample, the oracle's EM on the host-counted pattern
    histogram of every pair, every match_probability)."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings
    params = Params(cfg_settings(4, max_iterations=10), amd)
    st = params.settings
    job = Job("dedupe_only", [cfg4_records], "unique_id", 0, shard=shard)
    job.block(st["blocking_rules"])
    assert job.n_candidates > 2 ** 31 and job.n_pairs > 500_000_000
    job.gammas(st)
    if shard[1] == 8:
        check_shard(job, params, COLS, 10)
        return
    assert job.n_pairs > 2 ** 31 and job.ctx.gammas_windows() >= 2
    check_shard_streamed(job, params, COLS, 10)


CFG5_RULES = ["l.surname = r.surname", "l.dob = r.dob and l.city = r.city"]


def test_cfg5_shard_full_size(amd, heartbeat):
    """BASELINE configs[4] at one GPU's share: 100M records with the free-text address column (6 columns,
    address Levenshtein-4), pair-ordinal shard 0 of 8 (~1.21B of ~9.7e9 candidate pairs).  Blocking is
    surname | (dob AND city): surname | dob gives ~1.6e11 pairs at 100M records (29k dates put ~3,400
    records in each dob block), so the dob rule is narrowed by city to reach cfg5's ~1e10.
    Records: synthetic.make_records_parallel (64 chunks over one vocabulary).  A 2M-pair strided sample of
    comparison vectors bit-exact, 10 EM iterations and every match_probability at 1e-9 (README.md:14,
    case_statements.py:117-141)."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings, make_records_parallel
    cols = COLS + ["address"]
    df = make_records_parallel(100_000_000, 64, 16, surname_vocab=1_000_000, with_address=True)[["unique_id"] + cols]
    settings = cfg_settings(5, max_iterations=10)
    settings["blocking_rules"] = list(CFG5_RULES)
    params = Params(settings, amd)
    st = params.settings
    job = Job("dedupe_only", [df], "unique_id", 0, shard=(0, 8))
    del df
    job.block(st["blocking_rules"])
    assert job.n_candidates > 9_000_000_000 and job.n_pairs > 1_100_000_000
    job.gammas(st)
    check_shard(job, params, cols, 10)


@pytest.fixture(scope="module")
def cfg3_inputs():
    from splink_amd.synthetic import make_records_parallel
    df = make_records_parallel(20_000_000, 16, 16, surname_vocab=300_000)[["unique_id"] + COLS]
    return [df.iloc[:10_000_000].reset_index(drop=True), df.iloc[10_000_000:].reset_index(drop=True)]


def cfg3_job(amd, inputs, shard):
    """BASELINE configs[2]: link_only between two 10M-record tables (halves of one 20M population, so
    duplicates straddle them), rules surname | dob | email (~3.1e9 candidates, past 2^31), tf on surname;
    `shard` of its pair ordinals."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.synthetic import cfg_settings
    settings = cfg_settings(4, max_iterations=10)
    settings["link_type"] = "link_only"
    settings["blocking_rules"] = ["l.surname = r.surname", "l.dob = r.dob", "l.email = r.email"]
    for c in settings["comparison_columns"]:
        if c["col_name"] == "surname":
            c["term_frequency_adjustments"] = True
    params = Params(settings, amd)
    st = params.settings
    job = Job("link_only", inputs, "unique_id", 0, shard=shard)
    job.block(st["blocking_rules"])
    assert job.n_candidates > 2 ** 31
    job.gammas(st)
    return job, params


def surname_codes(job):
    """Host value codes of surname on both sides (device row order, -1 = NULL), one code space."""
    vl, vr = column_in_row_order(job, 0, "surname"), column_in_row_order(job, job.r_side(), "surname")
    codes, _ = pd.factorize(pd.concat([vl, vr], ignore_index=True), use_na_sentinel=True)
    return codes[:len(vl)], codes[len(vl):], int(codes.max()) + 1


def device_tf_table(job, params):
    """The product path's tf table on surname (term_frequencies.py's GPU stage): per-value Σmp and counts
    over the device dictionary ids, then bayes(adj_lambda, 1 - λ)."""
    from splink_amd.term_frequencies import _bayes_pair
    col = job._col_index[("surname", "str")]
    sums, counts = job.ctx.tf_accumulate_column(col, job.ctx.tf_column_values(col))
    with np.errstate(invalid="ignore", divide="ignore"):
        adj_lambda = np.where(counts > 0, sums / np.maximum(counts, 1), np.nan)
    return col, _bayes_pair(adj_lambda, float(1 - params.params["λ"]))


def test_cfg3_shard_full_size(amd, heartbeat, cfg3_inputs):
    """BASELINE configs[2] at one GPU's share of 8 (~386M pairs).  Comparison-vector sample, EM and
    match_probability as check_shard; then every pair's tf_adjusted_match_prob against oracle.tf_adjust_codes
    over host-factorised surnames at 1e-9 (blocking.py:95-160, term_frequencies.py:49-168)."""
    job, params = cfg3_job(amd, cfg3_inputs, (0, 8))
    assert job.n_pairs > 300_000_000
    mp, l, r = check_shard(job, params, COLS, 10)
    col, table = device_tf_table(job, params)
    tf_mp, _ = job.ctx.tf_apply_columns([col], [table], 0, job.n_pairs, want_adj=False)
    cl, cr, _ = surname_codes(job)
    want, _ = orc.tf_adjust_codes(cl[l], cr[r], mp, params.params["λ"])
    assert np.allclose(tf_mp, want, rtol=1e-9, atol=0, equal_nan=True)


@pytest.mark.timeout(900)
def test_cfg3_one_gpu_full_size(amd, heartbeat, cfg3_inputs):
    """BASELINE configs[2] whole on ONE GPU: ~3.09e9 link_only pairs in one context (past 2^31, so the
    comparison pass runs as ordinal windows), tf on surname.  check_shard_streamed (a 2M-pair strided sample
    of comparison vectors bit-exact, 10 EM iterations on the host-counted pattern histogram of every pair,
    every match_probability at 1e-9); then the per-value (Σmp, count) of equal-surname pairs accumulated on
    the host chunk by chunk over all pairs, and tf_adjusted_match_prob over 16 ranges spread across the
    ordinals (window edges included) at 1e-9 against oracle.tf_adjust_with_sums (term_frequencies.py:49-65,
    :122-168 have no size limit)."""
    job, params = cfg3_job(amd, cfg3_inputs, (0, 1))
    P = job.n_pairs
    assert P > 2 ** 31 and job.ctx.gammas_windows() >= 2
    check_shard_streamed(job, params, COLS, 10)
    cl, cr, n_v = surname_codes(job)
    lam = params.params["λ"]
    m_t, u_t = job.flat_tables(params._level_probabilities())
    sums, counts = np.zeros(n_v), np.zeros(n_v, dtype=np.int64)
    chunk = 1 << 27
    for c0 in range(0, P, chunk):  # the device's mp buffer is filled range by range, as on the host
        n = min(chunk, P - c0)
        mp = job.ctx.score(float(lam), float(1 - lam), m_t, u_t, c0, n)
        l, r = job.ctx.pairs_copy(c0, n)
        orc.tf_value_sums(cl[l], cr[r], mp, n_v, sums, counts)
        del mp, l, r
    col, table = device_tf_table(job, params)
    W = -(-P // job.ctx.gammas_windows())
    starts = sorted(set([int(x) for x in np.linspace(0, P - (1 << 20), 14)] + [max(0, W - (1 << 19))] +
                        [max(0, min(P - (1 << 20), 2 * W - (1 << 19)))]))
    for s0 in starts:
        n = min(1 << 20, P - s0)
        tf_mp, _ = job.ctx.tf_apply_columns([col], [table], s0, n, want_adj=False)
        mp = job.ctx.score(float(lam), float(1 - lam), m_t, u_t, s0, n)
        l, r = job.ctx.pairs_copy(s0, n)
        want, _ = orc.tf_adjust_with_sums(cl[l], cr[r], mp, lam, sums, counts)
        assert np.allclose(tf_mp, want, rtol=1e-9, atol=0, equal_nan=True), s0
