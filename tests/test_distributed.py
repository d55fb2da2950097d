"""N>1 host path on CPU: world_size-2 `gloo` ranks, pairs sharded by ordinal, one histogram all-reduce
per EM iteration (splink_amd.distributed, the code engine.Job.em_stats and bench.py use with RCCL).

Each rank takes the ordinal slice [P*r/W, P*(r+1)/W) of the candidate pairs (spk_block's shard rule,
spk_block.hip `g_lo/g_hi`), computes its comparison vectors and pattern histogram with the oracle,
and all-reduces the histogram.  The EM trajectory from the reduced histogram must equal the
single-process one, and the shards must partition the pair set.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as orc

SPECS = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]
COLS = ["first_name", "surname", "dob", "city", "email"]
NLEV = [3, 3, 2, 2, 3]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _workload():
    from splink_amd.synthetic import cfg_settings, make_records
    df = make_records(1500, seed=11, surname_vocab=80, first_vocab=120, city_vocab=40)[["unique_id"] + COLS]
    st = cfg_settings(1, max_iterations=6)
    pairs, left, right = orc.block(st, df=df)
    l = pairs["row_l"].to_numpy(np.int32)
    r = pairs["row_r"].to_numpy(np.int32)
    return left, right, l, r


def _gammas(left, right, l, r):
    cols_l = [orc.StrCol(left[c].tolist()) for c in COLS]
    cols_r = [orc.StrCol(right[c].tolist()) for c in COLS]
    return orc.template_gammas(SPECS, cols_l, cols_r, l, r)


def _codes(g):
    stride = np.cumprod([1] + [L + 1 for L in NLEV[:-1]])
    return ((g.astype(np.int64) + 1) * stride).sum(axis=1)


def _from_hist(hist):
    """The multiset of comparison vectors a histogram stands for (pattern order)."""
    stride = np.cumprod([1] + [L + 1 for L in NLEV[:-1]])
    pat = np.arange(len(hist))
    g = np.stack([(pat // s) % (L + 1) - 1 for s, L in zip(stride, NLEV)], axis=1).astype(np.int8)
    return np.repeat(g, hist, axis=0)


def _em(g):
    m0 = [[0.1, 0.2, 0.7], [0.1, 0.2, 0.7], [0.1, 0.9], [0.1, 0.9], [0.1, 0.2, 0.7]]
    u0 = [[0.7, 0.2, 0.1], [0.7, 0.2, 0.1], [0.9, 0.1], [0.9, 0.1], [0.7, 0.2, 0.1]]
    hist, _ = orc.em_iterate(g, NLEV, 0.3, m0, u0, 6, 1e-12)
    return hist


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splink_amd import distributed as D
    assert D.shard() == (rank, world)
    left, right, l, r = _workload()
    P = len(l)
    lo, hi = P * rank // world, P * (rank + 1) // world
    g = _gammas(left, right, l[lo:hi], r[lo:hi])
    n_pat = int(np.prod([L + 1 for L in NLEV]))
    hist = torch.from_numpy(np.bincount(_codes(g), minlength=n_pat).astype(np.int64))
    D.allreduce_histogram_(hist)
    total = D.sum_over_ranks(hi - lo)
    slowest = D.max_over_ranks(float(rank + 1))
    D.barrier()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), hist=hist.numpy(), total=total, slowest=slowest,
             lo=lo, hi=hi)
    dist.destroy_process_group()


def test_two_rank_gloo_em_matches_single_process(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [np.load(tmp_path / f"rank{k}.npz") for k in range(world)]
    left, right, l, r = _workload()
    # the shards partition the ordinal range
    assert res[0]["lo"] == 0 and res[0]["hi"] == res[1]["lo"] and res[1]["hi"] == len(l)
    for x in res:
        assert int(x["total"]) == len(l)
        assert float(x["slowest"]) == float(world)
    # every rank holds the same, full histogram
    g_full = _gammas(left, right, l, r)
    n_pat = int(np.prod([L + 1 for L in NLEV]))
    want = np.bincount(_codes(g_full), minlength=n_pat)
    assert (res[0]["hist"] == want).all() and (res[1]["hist"] == want).all()
    # and the EM trajectory from it is the single-process one
    h_single = _em(g_full)
    h_sharded = _em(_from_hist(res[0]["hist"]))
    assert len(h_single) == len(h_sharded)
    for (la, ma, ua), (lb, mb, ub) in zip(h_single, h_sharded):
        assert la == pytest.approx(lb, rel=1e-12)
        for a, b in zip(ma + ua, mb + ub):
            assert np.allclose(a, b, rtol=1e-12, atol=0)


def test_single_process_helpers_are_identity():
    from splink_amd import distributed as D
    assert D.shard() == (0, 1)
    assert D.sum_over_ranks(7) == 7 and D.max_over_ranks(2.5) == 2.5
    h = torch.arange(5)
    assert D.allreduce_histogram_(h) is h and h.tolist() == [0, 1, 2, 3, 4]


def _tf_rank_main(rank, world, port, out_dir):
    """Per-value (Σmp, count) tables of the tf adjustment summed over ranks (term_frequencies.py:49-65)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splink_amd import distributed as D
    rng = np.random.Generator(np.random.PCG64(3))
    ids = rng.integers(0, 50, 4000)           # value id of each pair (both sides equal)
    mp = rng.random(4000)
    lo, hi = 4000 * rank // world, 4000 * (rank + 1) // world
    sums = np.bincount(ids[lo:hi], weights=mp[lo:hi], minlength=50).astype(np.float64)
    counts = np.bincount(ids[lo:hi], minlength=50).astype(np.int64)
    # per-value scales (the exponent of each value's largest term) combine with MAX
    scale = np.full(50, np.iinfo(np.int32).min, dtype=np.int32)
    np.maximum.at(scale, ids[lo:hi], np.frexp(mp[lo:hi])[1].astype(np.int32))
    D.allreduce_host_(scale, op="max")
    D.allreduce_host_(sums)
    D.allreduce_host_(counts)
    np.savez(os.path.join(out_dir, f"tf{rank}.npz"), sums=sums, counts=counts, scale=scale)
    dist.destroy_process_group()


def test_two_rank_gloo_tf_tables(tmp_path):
    world = 2
    mp.start_processes(_tf_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    rng = np.random.Generator(np.random.PCG64(3))
    ids = rng.integers(0, 50, 4000)
    mpv = rng.random(4000)
    for k in range(world):
        x = np.load(tmp_path / f"tf{k}.npz")
        assert (x["counts"] == np.bincount(ids, minlength=50)).all()
        assert np.allclose(x["sums"], np.bincount(ids, weights=mpv, minlength=50), rtol=1e-12, atol=0)
        want = np.full(50, np.iinfo(np.int32).min, dtype=np.int32)
        np.maximum.at(want, ids, np.frexp(mpv)[1].astype(np.int32))
        assert np.array_equal(x["scale"], want)


def _gather_rank_main(rank, world, port, out_dir):
    """Replicated ingest (distributed.allgather_utf8_rows): each rank hands over its slice of the rows."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splink_amd import distributed as D
    arr = _gather_input()
    n, off, data, valid, on_dev = D.allgather_utf8_rows(arr)
    assert not on_dev
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), n=n, off=off, data=data, valid=valid)
    dist.destroy_process_group()


def _gather_input():
    import pyarrow as pa
    vals = ["ann", None, "", "bérénice", "o'brien", None, "z" * 300, "x"] * 251 + ["last"]
    return pa.array(["pad"] * 7 + vals, type=pa.large_string()).slice(7)  # a sliced array: offsets past 0


def test_two_rank_gloo_replicated_ingest(tmp_path):
    """Every rank of a two-rank job gets the whole column (offsets from 0, bytes, one validity byte per
    row) from the slices the ranks uploaded, identical to the column itself."""
    from splink_amd import table as T
    world = 2
    mp.start_processes(_gather_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    arr = _gather_input()
    off, data, bitmap, bit0 = T.arrow_views(arr)
    want_off = off - off[0]
    want_data = data[off[0]:off[-1]]
    want_valid = np.array([v is not None for v in arr.to_pylist()], dtype=np.uint8)
    for k in range(world):
        x = np.load(tmp_path / f"g{k}.npz")
        assert int(x["n"]) == len(arr)
        assert np.array_equal(x["off"], want_off)
        assert np.array_equal(x["data"][:len(want_data)], want_data)
        assert np.array_equal(x["valid"][:len(arr)], want_valid)
