"""A/B timing of comparison-vector pass variants on the bench workload (cfg2), one process."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from splink_amd.engine import Job
from splink_amd.params import Params
from splink_amd.session import AmdSession
from splink_amd.synthetic import cfg_settings, make_records
COLS = ["first_name", "surname", "dob", "city", "email"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
df = make_records(n, surname_vocab=int(os.environ.get("AB_VOCAB", "15000")), arrow=True)[["unique_id"] + COLS]
st = Params(cfg_settings(2), AmdSession(0)).settings
shard = tuple(int(x) for x in os.environ.get("AB_SHARD", "0/1").split("/"))
job = Job("dedupe_only", [df], "unique_id", 0, shard=shard)
job.ctx.enable_timing(True)
job.block(st["blocking_rules"])
ref = None
MODES = [int(m) for m in os.environ.get("AB_MODES", "1,2,1,2").split(",")]
for mode in MODES:
    job.ctx.gammas_set_simple(mode)
    job.gammas(st)
    ts = []
    for _ in range(5):
        job.gammas(st)
        ts.append(job.ctx.kernel_ms()["gamma"])
    g = job.gammas_host()
    if ref is None:
        ref = g
    cells = job.ctx.gammas_exact_counts(len(COLS))
    print(f"mode {mode}: gamma pass {np.median(ts):.3f} ms (min {min(ts):.3f}), same as first: {(g == ref).all()}, "
          f"exact cells {cells}", flush=True)
