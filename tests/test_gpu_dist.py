"""The RCCL (`nccl` backend) branch of the multi-GPU EM exchange, run on one GPU.

bench.py's N-GPU runs all-reduce the comparison-pattern histogram with RCCL between spk_em_histogram
(context stream) and spk_em_finalize (maximisation_step.py:36, 88 `collect()` of the GROUP BY in the
reference), and the term-frequency accumulators once per job (term_frequencies.py:84).  RCCL refuses
two ranks on one device, so here one rank opens a world-size-1 `nccl` group and forces both
collectives through dist.all_reduce on device tensors: the statistics must equal the one-launch
single-GPU iteration (spk_em_iteration) bit for bit, every iteration, with the parameters updated
in between (stream ordering between the context stream and torch's stream)."""
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

COLS = ["first_name", "surname", "dob", "city", "email"]


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist
    from splink_amd import _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    torch.cuda.set_device(0)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    yield dist
    dist.destroy_process_group()


def test_nccl_histogram_allreduce_matches_single_gpu(nccl_group):
    import torch
    from splink_amd import distributed as D
    from splink_amd.engine import Job, m_step_rows
    from splink_amd.params import Params
    from splink_amd.session import AmdSession
    from splink_amd.synthetic import cfg_settings, make_records
    assert nccl_group.get_backend() == "nccl"
    df = make_records(30000, seed=31, surname_vocab=600, first_vocab=400, city_vocab=100)[["unique_id"] + COLS]
    pa, pb = Params(cfg_settings(2, max_iterations=4), AmdSession(0)), Params(cfg_settings(2, max_iterations=4), AmdSession(0))
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(pa.settings["blocking_rules"])
    job.gammas(pa.settings)
    names, nlev = job.code_meta
    for _ in range(4):
        job.force_reduce = True   # histogram -> RCCL all-reduce (device tensor) -> finalize
        sa = job.em_stats(pa.params["λ"], pa._level_probabilities())
        job.force_reduce = False  # the one-launch iteration
        sb = job.em_stats(pb.params["λ"], pb._level_probabilities())
        assert np.array_equal(sa, sb)
        for p, st in ((pa, sa), (pb, sb)):
            lam, rows = m_step_rows(st, names, nlev)
            p._update_params(lam, rows)
    assert pa.params["λ"] == pb.params["λ"]
    # the host-staged all-reduce of the tf accumulators (int64) through RCCL is the identity at one rank
    arr = np.arange(-5, 1000, 7, dtype=np.int64).reshape(-1, 1) * np.int64(1 << 40)
    want = arr.copy()
    D.allreduce_host_(arr, force=True)
    assert np.array_equal(arr, want)
    # a device tensor reduced on torch's stream right after a context-stream kernel wrote it
    hist = torch.full((job.ctx.n_patterns(),), -7, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    job.ctx.em_histogram(hist.data_ptr())
    D.allreduce_histogram_(hist, force=True)
    torch.cuda.synchronize()
    assert int(hist.sum().item()) == job.n_pairs and int(hist.min().item()) >= 0


def test_nccl_stream_ordered_em_matches_single_gpu(nccl_group):
    """The N-GPU iteration with no host synchronisation (bench.py's pipelined multi-GPU step): the context
    moves onto a torch stream, spk_em_histogram_async -> dist.all_reduce on that stream (RCCL) ->
    spk_em_finalize_start, collected by em_wait while the next comparison pass is already queued.  The
    statistics equal the one-launch single-GPU iteration every iteration."""
    import copy

    from splink_amd.engine import Job, m_step_rows
    from splink_amd.params import Params
    from splink_amd.session import AmdSession
    from splink_amd.synthetic import cfg_settings, make_records
    df = make_records(30000, seed=32, surname_vocab=600, first_vocab=400, city_vocab=100)[["unique_id"] + COLS]
    st = cfg_settings(2, max_iterations=4)
    pa, pb = Params(copy.deepcopy(st), AmdSession(0)), Params(copy.deepcopy(st), AmdSession(0))
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.block(pa.settings["blocking_rules"])
    job.gammas(pa.settings)
    names, nlev = job.code_meta
    hist_a = []
    job.force_reduce = True
    pending = False
    for _ in range(4):  # pipelined, stream-ordered RCCL exchange
        job.gammas(pa.settings)
        if pending:
            s = job.em_wait()
            hist_a.append(s)
            pa._update_params(*m_step_rows(s, names, nlev))
        job.em_start(pa.params["λ"], pa._level_probabilities())
        pending = True
    s = job.em_wait()
    hist_a.append(s)
    pa._update_params(*m_step_rows(s, names, nlev))
    assert getattr(job, "_dist_stream", None) is not None
    job.force_reduce = False
    for i in range(4):  # one-launch iteration on the same context (now on the torch stream)
        job.gammas(pb.settings)
        s = job.em_stats(pb.params["λ"], pb._level_probabilities())
        assert np.array_equal(s, hist_a[i], equal_nan=True), i
        pb._update_params(*m_step_rows(s, names, nlev))
    assert pa.params["λ"] == pb.params["λ"]


def test_nccl_replicated_ingest_matches_local(nccl_group):
    """The replicated ingest's RCCL path (device all-gather of the rank's row slices, then the device copy
    into the raw columns) at world size 1: the encoded table (permutation, ranks, every comparison column,
    blocking keys) is byte-identical to a local ingest, and so are the pairs and comparison vectors."""
    from splink_amd.engine import Job
    from splink_amd.params import Params
    from splink_amd.session import AmdSession
    from splink_amd.synthetic import cfg_settings, make_records
    df = make_records(30000, seed=33, surname_vocab=600, first_vocab=400, city_vocab=100,
                      arrow=True)[["unique_id"] + COLS]
    st = Params(cfg_settings(2), AmdSession(0)).settings
    jobs = []
    for rep in (False, True):
        job = Job("dedupe_only", [df], "unique_id", 0, replicate=rep)
        assert job.replicate_ingest == rep
        job.block(st["blocking_rules"])
        job.gammas(st)
        jobs.append(job)
    a, b = jobs
    assert a.ctx.table_digest(0) == b.ctx.table_digest(0)
    la, ra = a.pair_rows()
    lb, rb = b.pair_rows()
    assert np.array_equal(la, lb) and np.array_equal(ra, rb)
    assert np.array_equal(a.gammas_host(), b.gammas_host())
