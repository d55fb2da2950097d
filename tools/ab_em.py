"""E+M iteration timings on the cfg2 workload's comparison vectors (one process): the one-launch
single-GPU iteration (spk_em_iteration) against its two-launch multi-GPU form (spk_em_histogram into a
device buffer + spk_em_finalize), both checked to give identical statistics.

    python tools/ab_em.py [records] [tile]    (tile > 1: the codes tiled that many times, as bench --em-scale)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from splink_amd.engine import N_HEAD, Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

COLS = ["first_name", "surname", "dob", "city", "email"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
tile = int(sys.argv[2]) if len(sys.argv) > 2 else 1
df = make_records(n, surname_vocab=15000, arrow=True)[["unique_id"] + COLS]
params = Params(cfg_settings(2), AmdSession(0))
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
hist = torch.empty(job.ctx.n_patterns(), dtype=torch.int64, device="cuda:0")
torch.cuda.synchronize()
out = {}
for rnd in range(2):
    for mode in ("fused", "split"):
        hs, fs = [], []
        for _ in range(10):
            if mode == "fused":
                stats = job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
            else:
                job.ctx.em_histogram(hist.data_ptr())
                stats = job.ctx.em_finalize(hist.data_ptr(), lam, 1 - lam, m, u, n_stats)
            ms = job.ctx.kernel_ms()
            hs.append(ms["em_hist"])
            fs.append(max(ms["em_final"], 0.0))
        out[mode] = stats
        print(f"{mode}: pairs {job.n_pairs}, histogram launch {np.median(hs) * 1e3:.1f} us, finalize launch "
              f"{np.median(fs) * 1e3:.1f} us", flush=True)
print("identical statistics:", bool((out["fused"] == out["split"]).all()))
