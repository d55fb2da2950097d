#!/bin/bash
# Round 3: exact-pass prologue in one round of independent loads (column descriptors, list bounds, first item and
# pair rows) -- full GPU tests, JW-launch timeline, cfg2 / cfg5 A/B against HEAD.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3ab.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3ab.log; tail -2 gpurun_out/tests_r3ab.log
[ $rc -ne 0 ] && exit $rc
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_xstamps.so timeout -k 10 300 python -u tools/ab_x_stamps.py 2>&1 | grep -v amdgpu.ids > gpurun_out/xstamps_r3ab.log || exit 1
cat gpurun_out/xstamps_r3ab.log
bash tools/gpu/ab_libs.sh "ab_head.so" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_head.so" || exit 1
echo done
