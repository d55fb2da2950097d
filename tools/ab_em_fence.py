"""E+M launch time with and without the agent-scope release fence before each workgroup's ticket
(spk_em_set_lane_histogram mode 1, the default, vs 2), on a bench workload's comparison vectors tiled x `tile`
(cfg2 or cfg5 columns), with identical statistics required.

    python tools/ab_em_fence.py [config] [tile]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
from splink_amd.engine import N_HEAD, Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
tile = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cols = ["first_name", "surname", "dob", "city", "email"] + (["address"] if cfg == 5 else [])
df = make_records(1_000_000, surname_vocab=15000, with_address=cfg == 5, arrow=True)[["unique_id"] + cols]
params = Params(cfg_settings(cfg), AmdSession(0))
st = params.settings
job = Job("dedupe_only", [df], "unique_id", 0)
job.ctx.enable_timing(True)
job.block(st["blocking_rules"])
job.gammas(st)
names, nlev = job.code_meta
if tile > 1:
    g = job.gammas_host()
    job.load_gammas(names, nlev, np.tile(g, (tile, 1)))
m, u = job.flat_tables(params._level_probabilities())
lam = params.params["λ"]
n_stats = N_HEAD + 4 * sum(L + 1 for L in nlev)
out = {}
for rnd in range(3):
    for mode in (1, 2):
        job.ctx.em_set_lane_histogram(mode)
        ts = []
        for _ in range(20):
            stats = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
            ts.append(job.ctx.kernel_ms()["em_hist"])
        out[mode] = stats
        if rnd:
            print(f"cfg{cfg} x{tile}: mode {mode} ({'fence' if mode == 1 else 'no fence'}): pairs {job.n_pairs}, "
                  f"E+M launch median {np.median(ts) * 1e3:.1f} us (min {min(ts) * 1e3:.1f})", flush=True)
print("identical statistics:", bool(np.array_equal(out[1], out[2])))
