#!/bin/bash
# Round 3: the filter's load groups (several row-image chunks per round trip) -- full GPU tests, then cfg2 A/B of
# pairs-per-lane / waves / chunks-per-group variants against HEAD, and cfg5 against HEAD.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3p.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3p.log; tail -2 gpurun_out/tests_r3p.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_head.so ab_f252.so ab_f244.so ab_f164.so ab_f243.so ab_f352.so" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_head.so" || exit 1
echo done
