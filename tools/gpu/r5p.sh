#!/bin/bash
# Round 5: the cfg5 100M-record share job with and without occupied-pattern ids (per-iteration E+M times).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
for v in nodense dense; do
  flag=""; [ $v = nodense ] && flag="--no-em-dense"
  timeout -k 10 400 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 \
    --workers 16 --rules "$RULES" --shard 0/8 --no-parity $flag --out gpurun_out/fj100M_r5p_$v.json \
    > gpurun_out/fj100M_r5p_$v.log 2>&1 || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/fj100M_r5p_$v.json'))
print('$v wall', round(d['job_wall_s'],3), 'em/iter', round(d['device_ms']['em_per_iter_mean'],4), d['device_ms']['em_per_iter'], d['em_dense_ids'])"
done
