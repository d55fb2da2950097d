#!/bin/bash
# Round 6: BASELINE configs[3] (20M-record dedupe) full jobs at its 2- and 8-GPU per-GPU shares on one GPU (no host
# parity pass: its host copies of ~3.1e9 pairs pass the box's host-memory cap; the -m gpu test
# test_cfg4_shard_full_size[0of2] holds that share's parity).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for sh in 0/8 0/2; do
  tag=${sh/\//of}
  timeout -k 10 600 python -u tools/full_job.py --config 4 --records 20000000 --surname-vocab 300000 --shard $sh \
    --chunks 16 --workers 16 --no-parity --out gpurun_out/r6_fulljob_cfg4_20M_shard$tag.json > gpurun_out/r6q_$tag.log 2>&1 \
    || { tail -20 gpurun_out/r6q_$tag.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r6_fulljob_cfg4_20M_shard$tag.json')); print('$sh', d['pairs_this_gpu'], d['job_wall_s'], d['device_ms']['gamma_pass'], d['device_ms']['em_per_iter_mean'], d['device_memory']['peak_in_use_bytes'])"
done
