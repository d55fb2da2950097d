#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_new.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "score or em_ or pipeline or edge or tf or sharded or scale" > gpurun_out/tests_abnew.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/tests_abnew.log; tail -2 gpurun_out/tests_abnew.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/abscore.log
for lib in A B A B; do
  if [ $lib == B ]; then export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_new.so; else unset SPLINK_AMD_LIB; fi
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 8 > gpurun_out/abscore_$lib.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/abscore_$lib.json')); e=d['em_at_scale']; b=d['breakdown_ms']
print('lib $lib', 'k_score %.4f ms frac %.3f' % (e['k_score']['avg_launch_ms'], e['k_score']['frac']), 'score@46M %.4f ms' % b['score'], 'headline %.3f' % d['hbm_headline_contract']['value'])" >> gpurun_out/abscore.log
done
cat gpurun_out/abscore.log
