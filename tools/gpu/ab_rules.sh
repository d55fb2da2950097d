#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_abrules -o run -- python -u tools/ab_rules.py > gpurun_out/ab_rules.log 2>&1 || exit 1
grep pairs gpurun_out/ab_rules.log
python - <<PY
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/prof_abrules/run_kernel_trace.csv")))
d = collections.defaultdict(list)
for r in rows:
    if "k_filter" in r["Kernel_Name"] or "exact_simple" in r["Kernel_Name"]:
        d[r["Kernel_Name"][:40]].append(round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1))
for k, v in d.items(): print(k, v)
PY
timeout -k 10 240 python -u tools/ab_em.py > gpurun_out/ab_em.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/ab_em.py 1000000 8 >> gpurun_out/ab_em.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/ab_em.log
