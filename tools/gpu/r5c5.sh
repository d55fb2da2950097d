#!/bin/bash
# Round 5 final: the cfg5 bench line (with its CPU baseline) on the final tree.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 --em-scale 0 > gpurun_out/bench_cfg5_r5c5.json 2> gpurun_out/bench_cfg5_r5c5.err || { tail -20 gpurun_out/bench_cfg5_r5c5.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_cfg5_r5c5.json')); a=d['string_rates']['levenshtein_exact_pass']['address']
print(d['value'], d['ms_per_step'], d['breakdown_ms']['gamma'], a['cells_compacted_out'], a['gcups_scanned'])"
