#!/bin/bash
# A/B of library builds on one box: parity subset per library, then bench.py alternating the in-tree
# library (A) and the candidates (splink_amd/ab_*.so, via SPLINK_AMD_LIB).
# Usage: bash tools/gpu/ab_libs.sh "ab_x.so ab_y.so" [pytest -k expression] [libraries to test, default "A";
# "skip": none]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}; K=${2:-"cfg2_full or simple_columns or case_levels or pipeline or levenshtein or jaro"}
TEST=${3:-A}
for lib in $TEST; do
  if [ $lib == skip ]; then continue; fi
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  tag=${lib//\//_}
  timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$K" > gpurun_out/tests_$tag.log 2>&1
  rc=$?; echo "$lib pytest exit $rc: $(tail -1 gpurun_out/tests_$tag.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
unset SPLINK_AMD_LIB
: > gpurun_out/ablibs.log
for rep in 1 2; do
  for lib in A $LIBS; do
    if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
    tag=${lib//\//_}
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --em-scale 0 ${BENCH_ARGS:-} > gpurun_out/ablib_$tag.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/ablib_$tag.json')); b=d['breakdown_ms']
print('$lib', 'ms/step %.4f' % d['ms_per_step'], 'gamma %.4f' % b['gamma'], 'em %.4f' % (b['em_hist'] + b['em_final']), 'em@scale %.3f' % d['em_at_scale']['em_iteration']['frac'] if d.get('em_at_scale') else '')" >> gpurun_out/ablibs.log
  done
done
cat gpurun_out/ablibs.log
