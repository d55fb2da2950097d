#!/bin/bash
# Round 3: full GPU tests with the gap-EQ filter loads and the two-level k_em_iter reduction; A/B of each
# against the previous commit's source (bench.py, same box).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3e.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3e.log; tail -2 gpurun_out/tests_r3e.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_oldfilter.so" "cfg2_full or simple_columns" || exit 1
bash tools/gpu/ab_score.sh "ab_oldem.so" || exit 1
echo done
