#!/bin/bash
# Round 3: M-step sums with half-wave slots and a DPP reduction tree, per-pattern globals written after the
# sums -- full GPU tests, stage stamps against HEAD, cfg2 A/B, HBM ceilings of plain streaming kernels.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3t.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3t.log; tail -2 gpurun_out/tests_r3t.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/stamps_r3t.log
for lib in ab_head_stamps.so ab_stamps.so; do
  echo "== $lib" >> gpurun_out/stamps_r3t.log
  SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib timeout -k 10 200 python -u tools/ab_em_stamps.py 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/stamps_r3t.log || exit 1
done
cat gpurun_out/stamps_r3t.log
bash tools/gpu/ab_libs.sh "ab_head.so" || exit 1
timeout -k 10 200 python -u tools/hbm_ceiling.py > gpurun_out/hbm_ceiling_r3t.json 2> gpurun_out/hbm_ceiling_r3t.err || exit 1
cat gpurun_out/hbm_ceiling_r3t.json
echo done
