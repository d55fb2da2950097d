#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5 -o run -- python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || exit 1
python -c "
import json,csv
d=json.load(open('gpurun_out/bench_cfg5.json'))
print('value',d['value'],'ms/step',d['ms_per_step'],'gamma',d['breakdown_ms']['gamma'], d['exact_cells_per_column'])
for r in csv.DictReader(open('gpurun_out/prof_cfg5/run_kernel_stats.csv')):
    if 'k_gamma' in r['Name']: print(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3)
"
