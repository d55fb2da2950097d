#!/bin/bash
# A/B of the E+M launch per library build: cfg2 and cfg5 bench lines with the at-scale E/M row (the run's
# codes tiled x8).  Usage: bash tools/gpu/ab_em.sh "ab_x.so ..."
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}
: > gpurun_out/abem.log
for cfg in 2 5; do
  for lib in A $LIBS; do
    if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
    tag=${lib//\//_}
    timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --em-scale 8 > gpurun_out/abem_${cfg}_$tag.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/abem_${cfg}_$tag.json')); b=d['breakdown_ms']; s=d.get('em_at_scale') or {}
e=s.get('em_iteration', {})
print('cfg$cfg $lib', 'ms/step %.4f' % d['ms_per_step'], 'em %.4f' % b['em_hist'], 'at-scale em %.4f ms frac %.3f' % (e.get('avg_launch_ms', -1), e.get('frac', -1)), 'pairs', s.get('pairs'))" >> gpurun_out/abem.log
  done
done
cat gpurun_out/abem.log
