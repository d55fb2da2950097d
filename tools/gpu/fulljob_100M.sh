#!/bin/bash
# cfg5 at its real per-GPU share: 100M records with the free-text address column, blocking
# surname | dob AND city (~1.2e10 candidate pairs), pair-ordinal shard 0 of 8 on one GPU; full job + parity.
# A 2M-record run of the same path first (quick check that the path works end to end).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 240 python -u tools/full_job.py --config 5 --records 2000000 --surname-vocab 20000 --chunks 8 --workers 8 \
  --rules "$RULES" --shard 0/1 --out gpurun_out/fulljob_cfg5_2M.json > gpurun_out/fulljob_cfg5_2M.log 2>&1 || exit 1
cat gpurun_out/fulljob_cfg5_2M.json
timeout -k 10 900 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 --workers 16 \
  --rules "$RULES" --shard 0/8 --out gpurun_out/fulljob_cfg5_100M.json > gpurun_out/fulljob_cfg5_100M.log 2>&1 || exit 1
cat gpurun_out/fulljob_cfg5_100M.json
