#!/bin/bash
# Parity tests, then the cfg2 bench + kernel trace and the cfg5 bench + kernel trace.  Usage: bash scripts_gpu_both.sh TAG
T=${1:-both}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_$T.log; tail -4 gpurun_out/tests_$T.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/benchprof_$T.json 2> gpurun_out/benchprof_$T.err || exit 1
bash scripts_gpu_cfg5.sh ${T}_c5 || exit 1
echo done
