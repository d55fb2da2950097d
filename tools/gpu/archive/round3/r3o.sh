#!/bin/bash
# Round 3: full GPU tests with one-gather JW fields and paired EQ fields, long free-text cells binned for the slow list; cfg2 / cfg5 A/B against HEAD.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3o.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3o.log; tail -2 gpurun_out/tests_r3o.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_head.so" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_head.so ab_nomark.so" || exit 1
echo done
