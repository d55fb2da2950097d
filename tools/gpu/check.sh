#!/bin/bash
# One GPU round-trip: parity tests, bench, rocprof kernel stats.  Usage: bash tools/gpu/check.sh TAG
# Stops at the first step that times out, aborts or faults (only plain test failures continue).
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 650 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_$TAG.log
tail -3 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err
echo "prof exit $?" >> gpurun_out/benchprof_$TAG.err
