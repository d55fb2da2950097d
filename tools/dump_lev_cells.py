"""Diagnostic: a random sample of the cells the filter hands to a Levenshtein exact pass (cfg2: email; cfg5: email
and address), written as JSON (strings and the pair's rows) for host analysis of the scans' trip counts.

    python tools/dump_lev_cells.py CONFIG OUT.json [cells]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from splink_amd.engine import Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

cfg, out = int(sys.argv[1]), sys.argv[2]
n_cells = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
cols = ["first_name", "surname", "dob", "city", "email"] + (["address"] if cfg == 5 else [])
df = make_records(1_000_000, surname_vocab=15000, with_address=cfg == 5, arrow=True)[["unique_id"] + cols]
st = Params(cfg_settings(cfg), AmdSession(0)).settings
job = Job("dedupe_only", [df], "unique_id", 0)
job.block(st["blocking_rules"])
job.ctx.gammas_set_lev_kernel(3)  # no character-bag decisions: every listed cell stays in the list
job.gammas(st)
names = job.code_meta[0]
cnt = job.ctx.gammas_exact_counts(len(names))
l, r = job.pair_rows()
t = job.tables[0]
rng = np.random.default_rng(0)
res = {"pairs": int(job.n_pairs), "exact_counts": dict(zip(names, [int(x) for x in cnt]))}
for k, name in enumerate(names):
    col = name.replace("gamma_", "")
    if col not in ("email", "address") or cnt[k] == 0:
        continue
    lst = job.ctx.gammas_exact_list(k, int(cnt[k]))
    lst = lst[lst >= 0]
    pick = lst[rng.choice(len(lst), min(n_cells, len(lst)), replace=False)]
    vals = t[col]
    res[col] = [[vals.iat[int(l[p])], vals.iat[int(r[p])]] for p in pick]
with open(out, "w") as f:
    json.dump(res, f)
print({k: (len(v) if isinstance(v, list) else v) for k, v in res.items()})
