#!/bin/bash
# One GPU round-trip: parity tests, bench, rocprof kernel stats, per-rule A/B, HBM traffic passes.
# Usage: bash scripts_gpu_round.sh TAG [skip-tests]
# Every GPU step has its own time limit; the script stops at the first step that times out,
# aborts or faults (plain test failures are recorded and the script goes on).
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
  rc=$?
  echo "pytest exit $rc" >> gpurun_out/tests_$TAG.log
  tail -3 gpurun_out/tests_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || exit 1
if [ -n "$AB" ]; then
  timeout -k 10 300 python -u tools/ab_rules.py 1000000 $AB > gpurun_out/abrules_$TAG.log 2>&1 || exit 1
  cat gpurun_out/abrules_$TAG.log
fi
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf_$TAG -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/pmcf_$TAG.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw_$TAG -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/pmcw_$TAG.log 2>&1 || exit 1
echo done
