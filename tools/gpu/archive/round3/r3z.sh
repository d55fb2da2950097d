#!/bin/bash
# Round 3: final score of the Myers scans from the diagonal helper; Levenshtein exact pass at 4 waves per SIMD
# (no spill) vs 5 -- full GPU tests, cfg2 / cfg5 A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3z.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3z.log; tail -2 gpurun_out/tests_r3z.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_head.so ab_lw4.so" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_head.so ab_lw4.so" || exit 1
echo done
