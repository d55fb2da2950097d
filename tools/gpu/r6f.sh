#!/bin/bash
# Round 6: cfg5 at the pair count of a 4-GPU job (100M records, pair-ordinal shard 0 of 4: ~2.4e9 pairs, two
# ordinal windows) on one GPU, no parity pass (test_cfg5_shard_full_size runs the 0/8 share's parity): the
# device-memory record by part -- does the 4-GPU layout fit 288 GB?  Then the 0/8 share as the round-6 record.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 900 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 --workers 16 \
  --rules "$RULES" --shard 0/4 --no-parity --out gpurun_out/r6_fulljob_cfg5_100M_shard0of4.json > gpurun_out/r6_fulljob_0of4.log 2>&1 || { tail -20 gpurun_out/r6_fulljob_0of4.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r6_fulljob_cfg5_100M_shard0of4.json')); print(d['pairs_this_gpu'], d['job_wall_s'], d['device_ms']['gamma_pass'], d['device_ms']['em_per_iter_mean']); print(json.dumps(d['device_memory']))"
