#!/bin/bash
# cfg5's columns at cfg5's per-GPU pair count: 20M records, shard 0/5 (~1.2B pairs), full job + parity.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
[ -n "$SKIP_SMALL" ] || timeout -k 10 300 python -u tools/full_job.py --config 5 --records 300000 --surname-vocab 4500 --shard 0/1 --out gpurun_out/fulljob_cfg5_small.json > gpurun_out/fulljob_cfg5_small.log 2>&1 || exit 1
[ -n "$SKIP_SMALL" ] || cat gpurun_out/fulljob_cfg5_small.json
timeout -k 10 1000 python -u tools/full_job.py --config 5 --records 20000000 --surname-vocab 300000 --shard 0/5 --out gpurun_out/fulljob_cfg5_20M.json > gpurun_out/fulljob_cfg5_20M.log 2>&1 || exit 1
cat gpurun_out/fulljob_cfg5_20M.json
