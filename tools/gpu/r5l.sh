#!/bin/bash
# Round 5: lane refill in the 128-bit slow pass -- parity subset, then the Levenshtein kernel A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "lev or cfg5 or exact_work or window or case_levels or pipeline or edge or strings_past or udf" \
  > gpurun_out/r5l_tests.log 2>&1 || { tail -40 gpurun_out/r5l_tests.log; exit 1; }
tail -1 gpurun_out/r5l_tests.log
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 0 2 1 2>&1 | grep -v amdgpu.ids > gpurun_out/r5l_ab.log || { cat gpurun_out/r5l_ab.log; exit 1; }
cat gpurun_out/r5l_ab.log
