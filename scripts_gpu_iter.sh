#!/bin/bash
# Iteration loop on the GPU box: parity tests, bench, kernel trace; PMC=1 adds SQ counter passes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-it}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_$T.log; tail -4 gpurun_out/tests_$T.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
cat gpurun_out/bench_$T.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/benchprof_$T.json 2> gpurun_out/benchprof_$T.err || exit 1
if [ -n "$PMC" ]; then
  pass() { local n=$1; shift; timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc${n}_$T -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc${n}_$T.log 2>&1; }
  pass 1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY || exit 1
  pass 2 SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum || exit 1
fi
echo done
