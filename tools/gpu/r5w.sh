#!/bin/bash
# Round 5: k_compact_lev with four list entries per thread -- Levenshtein / cfg5 tests, the cfg5 A/B, the cfg5
# kernel statistics.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r5w}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lev or cfg5 or address" \
  > gpurun_out/${TAG}_lev.log 2>&1 || { tail -40 gpurun_out/${TAG}_lev.log; exit 1; }
tail -1 gpurun_out/${TAG}_lev.log
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 3 2 2>&1 | grep -v amdgpu.ids > gpurun_out/${TAG}_ab.log || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_$TAG -o run -- python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2> gpurun_out/prof_cfg5_$TAG.err || exit 1
python3 - <<PY
import csv, glob
f = glob.glob('gpurun_out/prof_cfg5_$TAG/**/*kernel_stats.csv', recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
