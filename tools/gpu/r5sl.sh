#!/bin/bash
# Round 5: k_gamma_slow_lev at 4 waves per SIMD (128 VGPRs, spills) -- cfg5 kernel statistics and codes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r5sl}
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 4 3 2 2>&1 | grep -v amdgpu.ids > gpurun_out/${TAG}_ab.log || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_$TAG -o run -- python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2> gpurun_out/prof_cfg5_$TAG.err || exit 1
python3 - <<PY
import csv, glob
f = glob.glob('gpurun_out/prof_cfg5_$TAG/**/*kernel_stats.csv', recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:6]:
    print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
