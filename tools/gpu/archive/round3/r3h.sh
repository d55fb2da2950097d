#!/bin/bash
# Round 3: GPU tests with the M-step slot enumeration, E+M stage stamps, bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3h.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3h.log; tail -2 gpurun_out/tests_r3h.log
[ $rc -ne 0 ] && exit $rc
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_stamps.so timeout -k 10 200 python -u tools/ab_em_stamps.py > gpurun_out/em_stamps.log 2>&1 || exit 1
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_stamps.so timeout -k 10 200 python -u tools/ab_em_stamps.py 1000000 8 >> gpurun_out/em_stamps.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/em_stamps.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r3h.json 2>/dev/null || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bench_r3h.json')); b=d['breakdown_ms']; e=d['em_at_scale']
print('ms/step', d['ms_per_step'], 'gamma', b['gamma'], 'em', b['em_hist'], 'em@scale', e['em_iteration']['avg_launch_ms'], e['em_iteration']['frac'])"
echo done
