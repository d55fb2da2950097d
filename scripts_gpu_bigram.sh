#!/bin/bash
# Bigram-bound A/B and parity: new test + Levenshtein tests, then pass timings per filter variant.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "bigram or levenshtein or cfg5 or implied or view or simple_columns" > gpurun_out/tests_bigram.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/tests_bigram.log; tail -3 gpurun_out/tests_bigram.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AB_MODES=1,101,3,103,1,101 timeout -k 10 300 python -u tools/ab_gamma.py > gpurun_out/ab_bigram.log 2>&1 || exit 1
cat gpurun_out/ab_bigram.log
