#!/bin/bash
# A/B of library builds on the cfg5 columns (bench.py --config 5), alternating; parity via the cfg5 tests.
# Usage: bash tools/gpu/ab_cfg5.sh "ab_x.so ab_y.so"
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}
for lib in $LIBS; do
  SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "cfg5_address" > gpurun_out/tests_$lib.log 2>&1
  rc=$?; echo "$lib pytest exit $rc: $(tail -1 gpurun_out/tests_$lib.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
: > gpurun_out/abcfg5.log
for rep in 1 2; do
  for lib in A $LIBS; do
    if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
    timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 > gpurun_out/abcfg5_$lib.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/abcfg5_$lib.json')); b=d['breakdown_ms']
print('$lib', 'ms/step %.4f' % d['ms_per_step'], 'gamma %.4f' % b['gamma'])" >> gpurun_out/abcfg5.log
  done
done
cat gpurun_out/abcfg5.log
