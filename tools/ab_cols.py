"""Comparison-pass time per column subset of the cfg2 workload (one process; filter + exact passes).

    AB_SUBSETS="first_name,surname;dob,city;email" python tools/ab_cols.py [records]
"""
import copy
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
job.ctx.gammas_set_simple(int(os.environ.get("AB_MODE", "1")))
subsets = [s.split(",") for s in os.environ.get("AB_SUBSETS", ",".join(COLS) + ";first_name;surname;dob;city;email").split(";")]
for cols in subsets:
    s2 = copy.deepcopy(st)
    s2["comparison_columns"] = [c for c in st["comparison_columns"] if c["col_name"] in cols]
    job.gammas(s2)
    ts = []
    for _ in range(7):
        job.gammas(s2)
        ts.append(job.ctx.kernel_ms()["gamma"])
    print(f"{'+'.join(cols)}: pass {np.median(ts):.3f} ms, exact cells {job.ctx.gammas_exact_counts(len(cols))}",
          flush=True)
