#!/bin/bash
# A/B of E/M-at-scale kernels across library builds: bench.py's em_at_scale row (368M pairs) per library.
# Usage: bash tools/gpu/ab_score.sh "ab_x.so ab_y.so"
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}
: > gpurun_out/abscore.log
for rep in 1 2; do
  for lib in A $LIBS; do
    if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 8 > gpurun_out/abscore_$lib.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/abscore_$lib.json')); e=d['em_at_scale']
print('$lib', 'ms/step %.4f' % d['ms_per_step'], 'score %.4f ms frac %.3f' % (e['k_score']['avg_launch_ms'], e['k_score']['frac']),
      'em_iter %.4f ms frac %.3f' % (e['em_iteration']['avg_launch_ms'], e['em_iteration']['frac']))" >> gpurun_out/abscore.log
  done
done
cat gpurun_out/abscore.log
