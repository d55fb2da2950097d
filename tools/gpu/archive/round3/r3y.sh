#!/bin/bash
# Round 3: JW exact cells load both rows' planes with the records (one dependent gather round fewer) -- full
# GPU tests, cfg2 A/B against HEAD.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3y.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3y.log; tail -2 gpurun_out/tests_r3y.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_head.so" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3y -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
python - <<PY
import csv
for r in list(csv.DictReader(open("gpurun_out/prof_r3y/run_kernel_stats.csv")))[:10]: print(round(float(r["AverageNs"]) / 1e3, 1), "us x", r["Calls"], r["Name"][:70])
PY
echo done
