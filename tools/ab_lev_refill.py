"""Comparison pass time under the Levenshtein exact-pass kernels (spk_gammas_set_lev_kernel: 0 = one cell per
lane, 1 = lane refill everywhere, 2 = refill in free-text columns only) on a bench workload (cfg2 / cfg5 columns,
1M records), with identical codes required across all of them.  Reports the γ pass (device ms) and each column's
exact-pass launch time, medians of `reps`.

    python tools/ab_lev_refill.py [config] [reps] [mode ...]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
from splink_amd import _native as N  # noqa: E402
from splink_amd.engine import Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
variants = sys.argv[3:] or ["0", "1", "2"]
cols = ["first_name", "surname", "dob", "city", "email"] + (["address"] if cfg == 5 else [])
df = make_records(1_000_000, surname_vocab=15000, with_address=cfg == 5, arrow=True)[["unique_id"] + cols]
params = Params(cfg_settings(cfg), AmdSession(0))
st = params.settings
job = Job("dedupe_only", [df], "unique_id", 0)
job.ctx.enable_timing(True, exact=True)
job.block(st["blocking_rules"])
job.gammas(st)
names, nlev = job.code_meta
K = len(names)
lib = N.load_library()
stats = getattr(lib, "spk_debug_levq_stats", None)  # diagnostic build (-DSPK_LEVQ_STATS) only
STAT_NAMES = ["waves", "batches", "rounds", "handouts", "steps32", "steps64", "steps64long", "lane_steps/steps",
              "cells_scanned", "cyc_batches", "cyc_steps", "cyc_loop"]


def read_stats(reset=True):
    out = np.zeros(16, dtype=np.uint64)
    stats(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(1 if reset else 0))
    return out


codes = {}
for rnd in range(2):
    for v in variants:
        kern = int(v)
        job.ctx.gammas_set_lev_kernel(kern)
        if stats is not None:
            read_stats()
        g, x = [], []
        for _ in range(reps):
            job.gammas(st)
            g.append(job.ctx.kernel_ms()["gamma"])
            x.append(job.ctx.gammas_exact_ms(K))
        codes[v] = job.gammas_host()
        if stats is not None and kern > 0:
            d = dict(zip(STAT_NAMES, read_stats()[:12].tolist()))
            w = max(d["waves"], 1)
            print(f"  {v} schedule per wave ({d['waves']} waves): "
                  f"{ {k: round(val / w, 1) for k, val in d.items() if k != 'waves'} }", flush=True)
        if rnd:
            xm = np.median(np.array(x), axis=0)
            print(f"cfg{cfg} lev kernel {v}: pairs {job.n_pairs}, γ pass median {np.median(g):.3f} ms (min {min(g):.3f}); exact "
                  "launches ms " + ", ".join(f"{n} {val:.3f}" for n, val in zip(names, xm) if val >= 0), flush=True)
job.ctx.gammas_set_lev_kernel(2)
ref = codes[variants[0]]
print("identical codes:", all(bool(np.array_equal(ref, c)) for c in codes.values()))
