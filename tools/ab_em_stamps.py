"""Stage times of k_em_iter in the workgroup that finishes the reduction (diagnostic build):

    python tools/build_ab.py splink_amd/ab_stamps.so spk_em.hip -DSPK_EM_STAMPS
    SPLINK_AMD_LIB=splink_amd/ab_stamps.so python tools/ab_em_stamps.py [records] [tile]

Stamps (100 MHz wall clock): 0 block 0 starts, 1 the final workgroup starts, 2 it published its row,
3 its group's rows are all in (group ticket), 4 group row published, 5 all group rows in (final ticket),
6 group rows summed, 7 counts parked + arguments staged, 8 per-pattern E-step done, 9 M-step sums done."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd import _native as N  # noqa: E402
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
job.block(st["blocking_rules"])
job.gammas(st)
names, nlev = job.code_meta
if tile > 1:
    g = job.gammas_host()
    job.load_gammas(names, nlev, np.tile(g, (tile, 1)))
m, u = job.flat_tables(params._level_probabilities())
lam = params.params["λ"]
n_stats = N_HEAD + 4 * sum(L + 1 for L in nlev)
lib = N.load_library()
out = np.zeros(16, dtype=np.uint64)
rows = []
for it in range(12):
    job.ctx.em_iteration(lam, 1 - lam, m, u, n_stats)
    lib.spk_debug_em_stamps(out.ctypes.data_as(ctypes.c_void_p))
    if it >= 2:
        t = out.astype(np.int64)
        rows.append([(t[i] - t[0]) / 100.0 for i in range(10)])  # us from block 0's start
r = np.median(np.array(rows), axis=0)
names_ = ["block0 start", "final wg start", "own row published / streamed", "group complete / row adds", "group row published",
          "all groups in", "group rows summed", "args staged", "E-step per pattern", "M-step sums"]
print(f"pairs {job.n_pairs}: k_em_iter stages (median of {len(rows)}, us since block 0 started)")
for nm, x in zip(names_, r):
    print(f"  {nm:22s} {x:8.2f}")
