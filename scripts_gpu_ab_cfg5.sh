#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_new.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "levenshtein or cfg5 or strings or udf or lists" > gpurun_out/tests_abnew.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/tests_abnew.log; tail -2 gpurun_out/tests_abnew.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/abcfg5.log
for lib in A B A B; do
  if [ $lib == B ]; then export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_new.so; else unset SPLINK_AMD_LIB; fi
  timeout -k 10 200 python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > gpurun_out/abcfg5_$lib.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/abcfg5_$lib.json')); b=d['breakdown_ms']
print('lib $lib', 'value %.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'gamma %.3f' % b['gamma'])" >> gpurun_out/abcfg5.log
done
cat gpurun_out/abcfg5.log
