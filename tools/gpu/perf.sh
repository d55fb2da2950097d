#!/bin/bash
# Perf iteration: quick parity subset, bench line, rocprof kernel stats, one SQ counter pass.
# Usage: bash tools/gpu/perf.sh TAG [pytest -k expr]
TAG=${1:-perf}
K=${2:-"simple or blocking or cfg5 or levels or case_levels or pipeline or em_at_scale or cfg2_full"}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$K" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_$TAG.log
tail -3 gpurun_out/tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python - <<PY
import json; d=json.load(open("gpurun_out/bench_$TAG.json"))
print("value", d["value"], "ms/step", d["ms_per_step"], "breakdown", d["breakdown_ms"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || exit 1
python - <<PY
import csv,glob
f=glob.glob("gpurun_out/prof_$TAG/**/*kernel_stats.csv", recursive=True)[0]
rows=list(csv.DictReader(open(f)))
for r in rows[:14]: print(f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {r['Name'][:90]}")
PY
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pmc1_$TAG -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/pmc1_$TAG.log 2>&1 || exit 1
echo done
