#!/bin/bash
# Round 3: left rows shared within a wave in the filter (first lane of each run loads, ds_bpermute to the rest)
# -- full GPU tests, cfg2 and cfg5 A/B against HEAD.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3x.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3x.log; tail -2 gpurun_out/tests_r3x.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_head.so" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_head.so" || exit 1
echo done
