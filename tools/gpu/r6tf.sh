#!/bin/bash
# Round 6: the whole cfg3 job on one GPU with the tf histogram (mode 0) and the sort (mode 1), alternating.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for m in 0 1 0 1; do
  timeout -k 10 400 python -u tools/full_job.py --config 3 --records 10000000 --surname-vocab 300000 --shard 0/1 \
    --chunks 16 --workers 16 --no-parity --tf-mode $m --out gpurun_out/r6tf_m$m.json > gpurun_out/r6tf_m$m.log 2>&1 \
    || { tail -20 gpurun_out/r6tf_m$m.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r6tf_m$m.json')); w=d['wall_s']
print('mode $m', 'job %.3f' % d['job_wall_s'], 'tf_sums %.3f' % w['tf_sums'], 'tf_adjust %.3f' % w['tf_adjust'], 'block %.3f' % w['block'], 'score %.3f' % w['score'])" | tee -a gpurun_out/r6_ab_tf_hist.log
done
