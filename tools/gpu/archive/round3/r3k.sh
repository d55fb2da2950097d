#!/bin/bash
# Round 3: GPU tests with the LDS-staged left rows in the filter, A/B against the previous filter, kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3k.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3k.log; tail -2 gpurun_out/tests_r3k.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_nostage.so" "cfg2_full" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3k -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
python - <<PY
import csv
for r in list(csv.DictReader(open("gpurun_out/prof_r3k/run_kernel_stats.csv")))[:8]: print(round(float(r["AverageNs"]) / 1e3, 1), "us", r["Name"][:70])
PY
echo done
