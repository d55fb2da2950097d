#!/bin/bash
# Round 3: full GPU tests (k_em_iter parallel tail), filter-signature A/B without spills, kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3c.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3c.log; tail -3 gpurun_out/tests_r3c.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_libs.sh "ab_sig1w6.so ab_sig2w3.so" "cfg2_full or simple_columns or case_levels or pipeline" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3c -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/benchprof_r3c.json 2> gpurun_out/benchprof_r3c.err || exit 1
echo done
bash tools/gpu/ab_score.sh "ab_sc_u4w16t256.so ab_sc_u8w8t256.so ab_sc_u4w4t512.so" || exit 1
