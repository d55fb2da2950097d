"""Practical HBM ceilings on this GPU for the stream shapes of the E/M kernels, measured with torch's own
kernels (HIP events, 2.9 GB buffers): read-only (sum), write-only (fill), and 2 B read + 8 B write per
element (the k_score shape, as a gather-free index_select of an 8-byte table by 2-byte codes).  The
roofline fractions in bench.py use the 8 TB/s datasheet peak; these numbers say how much of that a
plain streaming kernel reaches here.

    python tools/hbm_ceiling.py [--gb 2.9] [--reps 20]
"""
import argparse
import json

import torch


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 1e3  # seconds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.9)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n8 = int(args.gb * 1e9) // 8
    x = torch.ones(n8, dtype=torch.float64, device=dev)
    out = {}
    t = timed(lambda: x.sum(), args.reps)
    out["read_only_sum_GBps"] = n8 * 8 / t / 1e9
    t = timed(lambda: x.fill_(1.5), args.reps)
    out["write_only_fill_GBps"] = n8 * 8 / t / 1e9
    y = torch.empty_like(x)
    t = timed(lambda: y.copy_(x), args.reps)
    out["copy_read_plus_write_GBps"] = 2 * n8 * 8 / t / 1e9
    codes = torch.randint(0, 576, (n8,), dtype=torch.int32, device=dev)
    table = torch.rand(576, dtype=torch.float64, device=dev)
    t = timed(lambda: torch.index_select(table, 0, codes, out=y), args.reps)
    out["gather_4B_in_8B_out_GBps"] = n8 * 12 / t / 1e9
    out["elements"] = n8
    out["peak_GBps_datasheet"] = 8000.0
    print(json.dumps(out))


if __name__ == "__main__":
    main()
