#!/bin/bash
# Round 5: bench.py smoke for cfg2 and cfg5 after the issue-counter source change.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in 2 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bq_cfg$c.json 2> gpurun_out/bq_cfg$c.err || { tail -20 gpurun_out/bq_cfg$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bq_cfg$c.json')); print('cfg$c', d['ms_per_step'], json.dumps(d['issue_gamma_kernels'])[:600])"
done
