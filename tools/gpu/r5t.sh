#!/bin/bash
# Round 5: character-bag decisions in every Levenshtein column (k_compact_lev) -- the
# Levenshtein / cfg5 tests, the A/B against mode 3 (no bag decisions), the cfg5 and cfg2 bench lines.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lev or cfg5 or address or windows" \
  > gpurun_out/r5t_lev.log 2>&1 || { tail -40 gpurun_out/r5t_lev.log; exit 1; }
tail -1 gpurun_out/r5t_lev.log
{ timeout -k 10 300 python -u tools/ab_lev_refill.py 2 6 3 2 && timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 3 2; } 2>&1 | grep -v amdgpu.ids > gpurun_out/r5t_ab.log || { cat gpurun_out/r5t_ab.log; exit 1; }
cat gpurun_out/r5t_ab.log
for c in 5 2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 > gpurun_out/bench_cfg${c}_r5t.json 2> gpurun_out/bench_cfg${c}_r5t.err || { tail -20 gpurun_out/bench_cfg${c}_r5t.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_cfg${c}_r5t.json'))
print('cfg$c', round(d['ms_per_step'],4), 'gamma', round(d['breakdown_ms']['gamma'],4), {k: (v['exact_cells'], v.get('bag_decided_cells'), round(v['exact_pass_ms'],3)) for k, v in d['string_rates']['levenshtein_exact_pass'].items()})"
done
