#!/bin/bash
# Round 3: JW exact cells in a JW-only kernel (120 VGPRs, 4 waves per SIMD instead of 2) -- full GPU tests,
# JW-launch timeline, cfg2 / cfg5 A/B against HEAD and the 5-wave (spilling) variant.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3ac.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3ac.log; tail -2 gpurun_out/tests_r3ac.log
[ $rc -ne 0 ] && exit $rc
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_xstamps.so timeout -k 10 300 python -u tools/ab_x_stamps.py 2>&1 | grep -v amdgpu.ids > gpurun_out/xstamps_r3ac.log || exit 1
head -12 gpurun_out/xstamps_r3ac.log
bash tools/gpu/ab_libs.sh "ab_head.so ab_jwc5.so" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_head.so" || exit 1
echo done
