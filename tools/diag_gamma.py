"""Diagnostic: where do device gammas differ from the oracle (at-scale synthetic data)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as orc
from splink_amd.engine import Job
from splink_amd.synthetic import cfg_settings, make_records
from splink_amd.settings import complete_settings_dict
from splink_amd.session import AmdSession
COLS = ["first_name", "surname", "dob", "city", "email"]
df = make_records(30000, seed=11, surname_vocab=800, first_vocab=400, city_vocab=100)[["unique_id"] + COLS]
st = complete_settings_dict(cfg_settings(2), AmdSession(0))
job = Job("dedupe_only", [df], "unique_id", 0)
job.block(st["blocking_rules"])
l, r = job.pair_rows()
t = job.tables[0]
specs = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]
cols = [orc.StrCol(t[c].tolist()) for c in COLS]
ref = orc.template_gammas(specs, cols, cols, l, r)
for simple in (True, False):
    job.ctx.gammas_set_simple(simple)
    job.gammas(st)
    gam = job.gammas_host()
    print("simple" if simple else "interp", "exact counts", job.ctx.gammas_exact_counts(5))
    for k, c in enumerate(COLS):
        bad = np.nonzero(gam[:, k] != ref[:, k])[0]
        print(f"  {c}: {len(bad)} mismatches")
        for i in bad[:6]:
            a, b = t[c][l[i]], t[c][r[i]]
            extra = orc.jaro_winkler(a, b) if k < 2 else (orc.levenshtein(a, b) if k == 4 else "")
            print(f"    {a!r} vs {b!r}: got {gam[i, k]} want {ref[i, k]} ({extra})")
