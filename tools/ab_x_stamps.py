"""Per-workgroup timeline of the JW exact launch (diagnostic build):

    python tools/build_ab.py splink_amd/ab_xstamps.so spk_gamma.hip -DSPK_X_STAMPS
    SPLINK_AMD_LIB=splink_amd/ab_xstamps.so python tools/ab_x_stamps.py

Prints when the workgroups start (dispatch timeline), how long working and empty ones live, and the
launch's span, all in us from the first workgroup's start (100 MHz wall clock)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from splink_amd import _native as N  # noqa: E402
from splink_amd.engine import Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

COLS = ["first_name", "surname", "dob", "city", "email"]
df = make_records(1_000_000, surname_vocab=15000, arrow=True)[["unique_id"] + COLS]
params = Params(cfg_settings(2), AmdSession(0))
st = params.settings
job = Job("dedupe_only", [df], "unique_id", 0)
job.block(st["blocking_rules"])
lib = N.load_library()
NB = 16384
out = np.zeros(5 * NB, dtype=np.uint64)
for it in range(4):
    job.gammas(st)
    job.ctx.synchronize() if hasattr(job.ctx, "synchronize") else None
    lib.spk_debug_x_stamps(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(5 * NB))
t = out.reshape(NB, 5).astype(np.int64)
used = t[:, 0] > 0
t = t[used]
t0 = t[:, 0].min()
start = (t[:, 0] - t0) / 100.0
end = (t[:, 1] - t0) / 100.0
dur = end - start
cells = t[:, 2]
work = cells > 0
print(f"workgroups {len(t)}, with cells {work.sum()}, span {end.max():.1f} us")
q = [0, 10, 50, 90, 100]
print("start us (percentiles 0/10/50/90/100):", np.percentile(start, q).round(1).tolist())
print("working wg duration us:", np.percentile(dur[work], q).round(1).tolist(), "iterations", np.percentile(cells[work], q).tolist())
if (~work).any():
    print("empty wg duration us:", np.percentile(dur[~work], q).round(1).tolist())
print("end us:", np.percentile(end, q).round(1).tolist())
w = t[work]
print("working wg: prologue (start -> after sync) us:", np.percentile((w[:, 3] - w[:, 0]) / 100.0, q).round(2).tolist())
print("working wg: first cell evaluated (after sync -> cell done) us:", np.percentile((w[:, 4] - w[:, 3]) / 100.0, q).round(2).tolist())
print("working wg: cell done -> end us:", np.percentile((w[:, 1] - w[:, 4]) / 100.0, q).round(2).tolist())
for lo in range(0, int(end.max()) + 10, 10):
    live = ((start <= lo + 10) & (end >= lo)).sum()
    print(f"  [{lo:3d},{lo + 10:3d}) us: started {((start >= lo) & (start < lo + 10)).sum():5d}  live {live:5d}")
