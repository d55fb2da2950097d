"""Multi-GPU plumbing: one process per GPU, candidate pairs sharded by ordinal, one exchange per EM iteration.

The reference's only cross-executor traffic on this path is Spark's shuffle of the partial
GROUP BY (maximisation_step.py:54-58) and the `collect()` of the tiny result (:36, :88).  Here
each rank holds the whole record table, generates only its slice of the global candidate-ordinal
space (spk_block shard / n_shards), and the only data-path collective is the all-reduce of the
comparison-pattern histogram (an exact integer sum, so every rank computes bit-identical
parameters whatever the rank count).  With the `nccl` backend that is RCCL over xGMI; with
`gloo` (CPU tests) the same code runs on host tensors.
"""
from __future__ import annotations


def _dist():
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover - torch always ships distributed on ROCm builds
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def shard() -> tuple:
    """(rank, world_size) of this process; (0, 1) without an initialised process group."""
    dist = _dist()
    if dist is None or dist.get_world_size() <= 1:
        return 0, 1
    return dist.get_rank(), dist.get_world_size()


def allreduce_histogram_(hist, force: bool = False):
    """In-place sum of a pattern histogram (int64 tensor, device or host) over all ranks.  force: run the
    collective even with one rank (tests exercise the RCCL path on a one-GPU box)."""
    dist = _dist()
    if dist is not None and (dist.get_world_size() > 1 or force):
        if hist.is_cuda and dist.get_backend() == "gloo":
            # gloo rehearsal of the multi-GPU path (several ranks on one device): host staging
            h = hist.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            hist.copy_(h)
        else:
            dist.all_reduce(hist, op=dist.ReduceOp.SUM)
    return hist


def stream_ordered_reduce(device: int) -> bool:
    """True when the histogram all-reduce can be queued on a device stream (backend nccl = RCCL), so the
    EM exchange needs no host synchronisation; False under gloo (host-staged rehearsal)."""
    dist = _dist()
    return dist is not None and dist.get_backend() != "gloo"


def allreduce_host_(arr, force: bool = False, op: str = "sum"):
    """In-place sum (op "sum") or maximum (op "max") over all ranks of a host numpy array (float64 / int64 /
    int32), e.g. the per-value fixed-point sums, counts and scales of the term-frequency adjustment
    (term_frequencies.py:49-65 groups over all pairs, which are sharded here).  RCCL needs device
    tensors, so under `nccl` the array is staged through the rank's GPU; under `gloo` it is reduced on
    the host."""
    import numpy as np
    import torch
    dist = _dist()
    if dist is None or (dist.get_world_size() <= 1 and not force) or arr.size == 0:
        return arr
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if dist.get_backend() != "gloo":
        t = t.to(f"cuda:{torch.cuda.current_device()}")
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    arr[...] = t.cpu().numpy()
    return arr


def _reduce_scalar(x, op, dtype):
    import torch
    dist = _dist()
    if dist is None or dist.get_world_size() <= 1:
        return x
    dev = "cpu" if dist.get_backend() == "gloo" else f"cuda:{torch.cuda.current_device()}"
    t = torch.tensor([x], dtype=dtype, device=dev)
    dist.all_reduce(t, op=op)
    return t.item()


def max_over_ranks(x: float) -> float:
    """Wall time of a step = the slowest rank's (bench.py contract)."""
    import torch
    dist = _dist()
    return float(_reduce_scalar(float(x), dist.ReduceOp.MAX if dist else None, torch.float64))


def sum_over_ranks(n: int) -> int:
    import torch
    dist = _dist()
    return int(_reduce_scalar(int(n), dist.ReduceOp.SUM if dist else None, torch.int64))


def barrier():
    dist = _dist()
    if dist is not None and dist.get_world_size() > 1:
        dist.barrier()


def allgather_utf8_rows(arr, force: bool = False):
    """Replicated ingest of one string column (the records are uploaded once and replicated
    over the ranks instead of every rank decoding the whole table from host memory): rank g hands over
    rows [g n / G, (g + 1) n / G) of the Arrow array, the ranks all-gather them -- RCCL over xGMI under
    `nccl` (device tensors), host tensors under `gloo` -- and every rank gets the whole column back.

    Returns (n, offsets, data, valid, on_device): int64 offsets [n + 1] from 0, the bytes, one validity byte
    per row; torch device tensors when on_device, else numpy arrays (Context.raw_utf8_device / _arrow)."""
    import numpy as np
    import torch
    from . import table as T
    dist = _dist()
    assert dist is not None and (dist.get_world_size() > 1 or force)
    rank, world = dist.get_rank(), dist.get_world_size()
    n = len(arr)
    lo, hi = n * rank // world, n * (rank + 1) // world
    off, data, bitmap, bit0 = T.arrow_views(arr.slice(lo, hi - lo))
    o = (off - off[0]).astype(np.int64)
    d = data[off[0]:off[-1]] if off[-1] > off[0] else np.zeros(0, np.uint8)
    if bitmap is None:
        v = np.ones(hi - lo, dtype=np.uint8)
    else:
        bits = np.unpackbits(bitmap, bitorder="little")
        v = bits[bit0: bit0 + (hi - lo)].astype(np.uint8)
    on_device = dist.get_backend() != "gloo"
    dev = torch.device(f"cuda:{torch.cuda.current_device()}") if on_device else torch.device("cpu")
    rows = [n * (g + 1) // world - n * g // world for g in range(world)]
    sz = torch.tensor([len(d)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, sz)
    sizes = [int(x.item()) for x in sizes]
    mb, mr = max(max(sizes), 1), max(rows)

    def gather(x, pad_to, dtype):
        t = torch.zeros(pad_to, dtype=dtype, device=dev)
        if len(x):
            t[:len(x)] = torch.from_numpy(np.ascontiguousarray(x)).to(dev)
        parts = [torch.empty(pad_to, dtype=dtype, device=dev) for _ in range(world)]
        dist.all_gather(parts, t)
        return parts

    dp = gather(d, mb, torch.uint8)
    op = gather(o[:-1], mr, torch.int64)
    vp = gather(v, mr, torch.uint8)
    base = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    offsets = torch.cat([op[g][:rows[g]] + int(base[g]) for g in range(world)] +
                        [torch.tensor([int(base[-1])], dtype=torch.int64, device=dev)])
    data_all = torch.cat([dp[g][:sizes[g]] for g in range(world)] + [torch.zeros(1, dtype=torch.uint8, device=dev)])
    valid = torch.cat([vp[g][:rows[g]] for g in range(world)] + [torch.zeros(1, dtype=torch.uint8, device=dev)])
    if on_device:
        torch.cuda.synchronize(dev)  # the context reads them on its own stream
        return n, offsets, data_all, valid, True
    return n, offsets.numpy(), data_all.numpy(), valid.numpy(), False
