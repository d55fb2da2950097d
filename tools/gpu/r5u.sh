#!/bin/bash
# Round 5: the full GPU suite after the character-bag decisions (free-text columns) and the sampled E+M
# pattern, the cfg5 A/B, the cfg5 / cfg2 bench lines, the cfg5 100M-record share job.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5u_suite.log 2>&1 || { tail -30 gpurun_out/r5u_suite.log; exit 1; }
tail -1 gpurun_out/r5u_suite.log
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 3 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r5u_ab.log || { cat gpurun_out/r5u_ab.log; exit 1; }
cat gpurun_out/r5u_ab.log
for c in 5 2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 > gpurun_out/bench_cfg${c}_r5u.json 2> gpurun_out/bench_cfg${c}_r5u.err || { tail -20 gpurun_out/bench_cfg${c}_r5u.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg${c}_r5u.json'))
print('cfg$c', round(d['ms_per_step'],4), 'gamma', round(d['breakdown_ms']['gamma'],4), {k: (v['exact_cells'], v.get('cells_compacted_out'), round(v['exact_pass_ms'],3)) for k, v in d['string_rates']['levenshtein_exact_pass'].items()})"
done
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 400 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 \
  --workers 16 --rules "$RULES" --shard 0/8 --no-parity --out gpurun_out/fj100M_r5u.json \
  > gpurun_out/fj100M_r5u.log 2>&1 || exit 1
python -c "
import json; d=json.load(open('gpurun_out/fj100M_r5u.json'))
print('wall', round(d['job_wall_s'],3), 'em/iter', round(d['device_ms']['em_per_iter_mean'],4), 'gamma', round(d['device_ms']['gamma_pass'],2), {k: round(v,3) for k,v in d['wall_s'].items()})"
