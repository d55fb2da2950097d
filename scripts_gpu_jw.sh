#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "jaro or udf or case_levels or scale or pipeline or simple_columns or strings" > gpurun_out/tests_jw.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/tests_jw.log; tail -2 gpurun_out/tests_jw.log
if [ $rc -ne 0 ]; then exit $rc; fi
AB_MODES=1,3000001,1,3000001 timeout -k 10 300 python -u tools/ab_gamma.py > gpurun_out/ab_jw.log 2>&1 || exit 1
grep mode gpurun_out/ab_jw.log
