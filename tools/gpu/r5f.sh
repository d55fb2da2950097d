#!/bin/bash
# Round 5: the GPU suite on the single-tier E+M kernel, the fence A/B (tools/ab_em_fence.py) at cfg2 / cfg5,
# and the cfg5 100M-record share job (E+M per iteration at the real pattern concentration).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5f_suite.log 2>&1 || { tail -30 gpurun_out/r5f_suite.log; exit 1; }
tail -3 gpurun_out/r5f_suite.log
timeout -k 10 300 python -u tools/ab_em_fence.py 2 8 > gpurun_out/r5f_fence.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_em_fence.py 5 4 >> gpurun_out/r5f_fence.log 2>&1 || exit 1
cat gpurun_out/r5f_fence.log
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 400 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 \
  --workers 16 --rules "$RULES" --shard 0/8 --no-parity --out gpurun_out/fj100M_r5f.json \
  > gpurun_out/fj100M_r5f.log 2>&1 || exit 1
python -c "
import json; d=json.load(open('gpurun_out/fj100M_r5f.json'))
print('wall', round(d['job_wall_s'],3), 'em/iter', round(d['device_ms']['em_per_iter_mean'],4), 'gamma', round(d['device_ms']['gamma_pass'],2), {k: round(v,3) for k,v in d['wall_s'].items()})"
