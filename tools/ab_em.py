"""A/B of the E/M histogram variants on the cfg2 workload's comparison vectors (one process).

    AB_HIST=1,0,1,0 python tools/ab_em.py [records]
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
params = Params(cfg_settings(2), AmdSession(0))
st = params.settings
job = Job("dedupe_only", [df], "unique_id", 0)
job.ctx.enable_timing(True)
job.block(st["blocking_rules"])
job.gammas(st)
ref = None
for mode in [int(x) for x in os.environ.get("AB_HIST", "1,0,1,0").split(",")]:
    job.ctx.em_set_lane_histogram(mode)
    hs, fs = [], []
    for _ in range(12):
        stats = job.em_stats(params.params["λ"], params._level_probabilities())
        ms = job.ctx.kernel_ms()
        hs.append(ms["em_hist"])
        fs.append(ms["em_final"])
    ref = stats if ref is None else ref
    print(f"hist mode {mode}: em_hist {np.median(hs) * 1e3:.1f} us (min {min(hs) * 1e3:.1f}), em_final "
          f"{np.median(fs) * 1e3:.1f} us, same stats: {bool((np.asarray(stats) == np.asarray(ref)).all())}", flush=True)
