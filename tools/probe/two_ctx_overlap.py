"""Probe: do two comparison passes on two contexts (two HIP streams) overlap on one GPU?  cfg2 (1M records),
20 passes of one job alone, then 20 rounds of two jobs' passes queued back to back (each job on its own
context stream).  If a round takes well under two passes, the filter (texture-address bound) and the
Levenshtein / JW exact passes (VALU / latency bound) of different passes share the CUs usefully."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from splink_amd.engine import Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

cols = ["first_name", "surname", "dob", "city", "email"]
df = make_records(1_000_000, surname_vocab=15000, arrow=True)[["unique_id"] + cols]
st = Params(cfg_settings(2), AmdSession(0)).settings
jobs = [Job("dedupe_only", [df], "unique_id", 0) for _ in range(2)]
for j in jobs:
    j.block(st["blocking_rules"])
    j.gammas(st)
    j.gammas_host()
N = 20
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        jobs[0].gammas(st)
    jobs[0].gammas_host() if rep < 0 else None
    torch.cuda.synchronize()
    one = (time.perf_counter() - t0) / N * 1e3
    t0 = time.perf_counter()
    for _ in range(N):
        jobs[0].gammas(st)
        jobs[1].gammas(st)
    torch.cuda.synchronize()
    two = (time.perf_counter() - t0) / N * 1e3
    print(f"one pass {one:.3f} ms, two passes on two streams {two:.3f} ms per round ({two / one:.2f} x one)", flush=True)
a = jobs[0].gammas_host()
b = jobs[1].gammas_host()
print("codes identical:", bool((a == b).all()))
