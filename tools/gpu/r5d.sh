#!/bin/bash
# Round 5: cfg2 and cfg5 bench lines with kernel statistics (rocprofv3 --kernel-trace --stats).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r5d}
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json | python -c "import json,sys; d=json.load(sys.stdin); print('cfg2', d['value'], d['ms_per_step'], d['breakdown_ms']['gamma'], d['breakdown_ms']['em_hist'], (d.get('em_at_scale') or {}).get('em_iteration',{}).get('frac'))"
timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 > gpurun_out/bench_cfg5_$TAG.json 2> gpurun_out/bench_cfg5_$TAG.err || exit 1
cat gpurun_out/bench_cfg5_$TAG.json | python -c "import json,sys; d=json.load(sys.stdin); print('cfg5', d['value'], d['ms_per_step'], d['breakdown_ms']['gamma'], d['breakdown_ms']['em_hist'], (d.get('em_at_scale') or {}).get('em_iteration',{}).get('frac'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_$TAG -o run -- python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2> gpurun_out/prof_cfg5_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2> gpurun_out/prof_$TAG.err || exit 1
find gpurun_out/prof_cfg5_$TAG gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head
