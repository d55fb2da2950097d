#!/bin/bash
# Round 5: hot-pattern sampling before the first E+M launch on a pair set -- the E/M tests, the bench lines,
# the cfg5 100M-record share job (per-iteration E+M times).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "em_ or test_em" \
  > gpurun_out/r5q_em.log 2>&1 || { tail -40 gpurun_out/r5q_em.log; exit 1; }
tail -1 gpurun_out/r5q_em.log
for c in 2 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 > gpurun_out/bench_cfg${c}_r5q.json 2> gpurun_out/bench_cfg${c}_r5q.err || { tail -20 gpurun_out/bench_cfg${c}_r5q.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg${c}_r5q.json'))
e=d['em_at_scale']; print('cfg$c', round(d['ms_per_step'],4), 'em', round(d['phase_ms']['em'],4) if 'phase_ms' in d else '', 'at-scale em', round(e['em_iteration']['avg_launch_ms'],4), 'frac', round(e['em_iteration']['frac'],3))"
done
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 400 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 \
  --workers 16 --rules "$RULES" --shard 0/8 --no-parity --out gpurun_out/fj100M_r5q.json \
  > gpurun_out/fj100M_r5q.log 2>&1 || exit 1
python -c "
import json; d=json.load(open('gpurun_out/fj100M_r5q.json'))
print('wall', round(d['job_wall_s'],3), 'em/iter', round(d['device_ms']['em_per_iter_mean'],4), d['device_ms']['em_per_iter'], d['pattern_concentration'])"
