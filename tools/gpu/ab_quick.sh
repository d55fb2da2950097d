#!/bin/bash
# Quick A/B timings: the filter with / without the rule-view launch, the E+M iteration forms.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
AB_MODES=${AB_MODES:-11,21,11,21} timeout -k 10 240 python -u tools/ab_gamma.py > gpurun_out/ab_views.log 2>&1 || exit 1
cat gpurun_out/ab_views.log
timeout -k 10 240 python -u tools/ab_em.py > gpurun_out/ab_em.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/ab_em.py 1000000 8 >> gpurun_out/ab_em.log 2>&1 || exit 1
cat gpurun_out/ab_em.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_abem -o run -- python -u tools/ab_em.py > gpurun_out/prof_abem.log 2>&1 || exit 1
python - <<PY
import csv, glob
f = glob.glob("gpurun_out/prof_abem/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {r['Name'][:90]}")
PY
