"""Where the comparison pass spends its time, by blocking rule (cfg2 workload, one process).

Times the comparison-vector pass over (a) every pair, (b) only the pairs of rule 0 (`surname`,
whose blocks are contiguous in the clustered table), (c) only the pairs of rule 1 (`dob`, whose
rows are scattered over the table), and (d) the same dob pairs when the table is clustered by dob
instead -- the gain a rule-local row order would give the second rule.
"""
import os
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd.engine import Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

COLS = ["first_name", "surname", "dob", "city", "email"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
modes = [int(m) for m in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2]
df = make_records(n, surname_vocab=15000)[["unique_id"] + COLS]
st = Params(cfg_settings(2), AmdSession(0)).settings


def timed(job, label, reps=5):
    job.gammas(st)
    ts = []
    for _ in range(reps):
        job.gammas(st)
        ts.append(job.ctx.kernel_ms()["gamma"])
    ex = dict(zip(job.code_meta[0], job.ctx.gammas_exact_counts(len(job.code_meta[0]))))
    med = float(np.median(ts))
    print(f"{label:44s} pairs {job.n_pairs:>10d}  gamma pass {med:7.3f} ms  "
          f"({job.n_pairs / med / 1e6:6.2f} Gpairs/s)  exact {ex}", flush=True)


for mode in modes:
    print(f"--- filter mode {mode} (1 = per-column gathers, 2 = register rows)", flush=True)
    job = Job("dedupe_only", [df], "unique_id", 0)
    job.ctx.enable_timing(True)
    job.ctx.gammas_set_simple(mode)
    job.block(st["blocking_rules"])
    l, r = job.pair_rows()
    t = job.tables[0]
    sn = t["surname"].to_numpy()
    ok = pd.notna(t["surname"]).to_numpy()
    rule0 = ok[l] & (sn[l] == sn[r])
    n0 = int(rule0.sum())
    assert rule0[:n0].all() and not rule0[n0:].any(), "pairs are not rule-major"
    timed(job, "all pairs (surname-clustered table)")
    job.load_pairs(l[:n0], r[:n0])
    timed(job, "rule 0 (surname) pairs")
    job.load_pairs(l[n0:], r[n0:])
    timed(job, "rule 1 (dob) pairs, scattered rows")

    job2 = Job("dedupe_only", [df], "unique_id", 0)
    job2.ctx.enable_timing(True)
    job2.ctx.gammas_set_simple(mode)
    job2.block(["l.dob = r.dob", "l.surname = r.surname"])
    l2, r2 = job2.pair_rows()
    t2 = job2.tables[0]
    dob = t2["dob"].to_numpy()
    okd = pd.notna(t2["dob"]).to_numpy()
    sn2 = t2["surname"].to_numpy()
    oks = pd.notna(t2["surname"]).to_numpy()
    # the pairs rule 1 of the first job emitted: equal dob and not equal surname
    keep = okd[l2] & (dob[l2] == dob[r2]) & ~(oks[l2] & (sn2[l2] == sn2[r2]))
    job2.load_pairs(l2[keep], r2[keep])
    timed(job2, "rule 1 (dob) pairs, dob-clustered rows")
