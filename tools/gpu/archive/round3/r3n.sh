#!/bin/bash
# Round 3: full GPU tests with the early bounce of long free-text cells; cfg5 A/B against the previous build.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3n.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3n.log; tail -2 gpurun_out/tests_r3n.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_cfg5.sh "ab_nobounce.so" || exit 1
bash tools/gpu/ab_score.sh "ab_sc_u8.so ab_sc_u2.so ab_sc_wg16.so ab_sc_wg4.so ab_sc_t1024.so" || exit 1
echo done
