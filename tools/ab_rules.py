"""Comparison-pass time on each blocking rule's pairs alone (cfg2 workload, one process): the pairs of
rule 0 (surname blocks: rows contiguous in the clustered table) against those of rule 1 (dob blocks:
rows scattered), loaded with spk_pairs_load so the filter sees each set on its own.

    python tools/ab_rules.py [records]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd.engine import Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

COLS = ["first_name", "surname", "dob", "city", "email"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
df = make_records(n, surname_vocab=15000, arrow=True)[["unique_id"] + COLS]
st = Params(cfg_settings(2), AmdSession(0)).settings
job = Job("dedupe_only", [df], "unique_id", 0)
job.ctx.enable_timing(True)
job.block(st["blocking_rules"])
l, r = job.pair_rows()
t = job.tables[0]
sn = t["surname"].to_numpy(dtype=object, na_value=None)
rule0 = np.array([a is not None and a == b for a, b in zip(sn[l], sn[r])], dtype=bool)
n0 = int(rule0.sum())
assert rule0[:n0].all() and not rule0[n0:].any()
sets = {"all": (l, r), "rule0": (l[:n0], r[:n0]), "rule1": (l[n0:], r[n0:]),
        "rule1_sorted": tuple(x[n0:][np.lexsort((r[n0:], l[n0:]))] for x in (l, r))}
for rnd in range(2):
    for name, (a, b) in sets.items():
        job.load_pairs(a, b)
        job.gammas(st)
        ts = []
        for _ in range(5):
            job.gammas(st)
            ts.append(job.ctx.kernel_ms()["gamma"])
        print(f"{name}: {len(a)} pairs, gamma pass {np.median(ts):.3f} ms, {len(a) / np.median(ts) / 1e6:.3f} Gpairs/s, "
              f"exact cells {job.ctx.gammas_exact_counts(len(COLS))}", flush=True)
