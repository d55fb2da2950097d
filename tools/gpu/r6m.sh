#!/bin/bash
# Round 6: cfg5 at its 100M-record 0/8 share (1.21e9 pairs on one GPU) with the two-stream split (default) and the
# one-stream pass timed beside it, no parity pass (test_cfg5_shard_full_size runs the parity with the same default).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 900 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 --workers 16 \
  --rules "$RULES" --shard 0/8 --no-parity --out gpurun_out/r6_fulljob_cfg5_100M_shard0of8.json > gpurun_out/r6_fulljob_0of8.log 2>&1 || { tail -20 gpurun_out/r6_fulljob_0of8.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r6_fulljob_cfg5_100M_shard0of8.json')); print(d['pairs_this_gpu'], d['job_wall_s'], d['device_ms']); print(json.dumps(d.get('device_memory'))[:600])"
