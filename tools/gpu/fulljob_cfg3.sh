#!/bin/bash
# cfg3 (link_only 2 x N + tf on surname): tf parity tests, a small full job, then the per-GPU share of 2 x 10M.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "tf or link" > gpurun_out/tests_cfg3.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/tests_cfg3.log; tail -2 gpurun_out/tests_cfg3.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/full_job.py --config 3 --records 200000 --surname-vocab 3000 --shard 0/1 --out gpurun_out/fulljob_cfg3_small.json > gpurun_out/fulljob_cfg3_small.log 2>&1 || exit 1
cat gpurun_out/fulljob_cfg3_small.json
if [ "$1" == "big" ]; then
  timeout -k 10 900 python -u tools/full_job.py --config 3 --records 10000000 --surname-vocab 300000 --shard 0/8 --out gpurun_out/fulljob_cfg3_10M.json > gpurun_out/fulljob_cfg3_10M.log 2>&1 || exit 1
  cat gpurun_out/fulljob_cfg3_10M.json
fi
