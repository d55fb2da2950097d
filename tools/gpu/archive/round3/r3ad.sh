#!/bin/bash
# Round 3 end: cfg4's per-GPU share full job (20M records, shard 0/8) and the 2M-record cfg5 job with the final
# exact-pass code, parity legs included.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/full_job.py --records 20000000 --shard 0/8 --out gpurun_out/fulljob_cfg4_r3ad.json > gpurun_out/fulljob_cfg4_r3ad.log 2>&1 || exit 1
python -c "
import json; d=json.load(open('gpurun_out/fulljob_cfg4_r3ad.json')); print('cfg4', d.get('pairs_this_gpu'), d.get('job_wall_s'), d.get('parity_gamma'), d.get('parity_em'))"
timeout -k 10 600 python -u tools/full_job.py --config 5 --records 2000000 --out gpurun_out/fulljob_cfg5_2M_r3ad.json > gpurun_out/fulljob_cfg5_2M_r3ad.log 2>&1 || exit 1
python -c "
import json; d=json.load(open('gpurun_out/fulljob_cfg5_2M_r3ad.json')); print('cfg5 2M', d.get('pairs_this_gpu'), d.get('job_wall_s'), d.get('parity_gamma'), d.get('parity_em'))"
echo done
