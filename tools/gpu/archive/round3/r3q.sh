#!/bin/bash
# Round 3: free-text Levenshtein cells with rows past 64 units binned on their own (cfg5): full GPU tests, cfg5 and
# cfg2 A/B against HEAD.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3q.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3q.log; tail -2 gpurun_out/tests_r3q.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_cfg5.sh "ab_head.so" || exit 1
bash tools/gpu/ab_libs.sh "ab_head.so" || exit 1
echo done
