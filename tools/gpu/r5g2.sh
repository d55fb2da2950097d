#!/bin/bash
# Round 5 final: the full GPU suite on the final tree and the cfg5 100M-record share job.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5g2_suite.log 2>&1 || { tail -30 gpurun_out/r5g2_suite.log; exit 1; }
tail -1 gpurun_out/r5g2_suite.log
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 400 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 \
  --workers 16 --rules "$RULES" --shard 0/8 --no-parity --out gpurun_out/fj100M_r5g2.json \
  > gpurun_out/fj100M_r5g2.log 2>&1 || exit 1
python -c "
import json; d=json.load(open('gpurun_out/fj100M_r5g2.json'))
print('wall', round(d['job_wall_s'],3), 'em/iter', round(d['device_ms']['em_per_iter_mean'],4), 'gamma', round(d['device_ms']['gamma_pass'],2), {k: round(v,3) for k,v in d['wall_s'].items()})"
