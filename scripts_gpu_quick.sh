#!/bin/bash
# Quick GPU check: string-kernel parity subset, then bench + rocprof kernel stats.  Usage: bash scripts_gpu_quick.sh TAG [pytest -k expr]
TAG=${1:-quick}
K=${2:-"levenshtein or cfg5 or scale or strings or udf or view or simple_columns or implied or lists"}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$K" > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/tests_$TAG.log; tail -3 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python -c "
import json,csv
d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value',d['value'],'ms/step',d['ms_per_step'],'gamma',d['breakdown_ms']['gamma'])
for r in csv.DictReader(open('gpurun_out/prof_$TAG/run_kernel_stats.csv')):
    if 'k_gamma' in r['Name'] or 'k_hist' in r['Name']: print(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3)
"
