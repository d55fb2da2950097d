#!/bin/bash
# Round 5: the lane-refill Levenshtein exact kernel -- Levenshtein parity tests, then the A/B against the
# one-cell-per-lane kernel at cfg2 / cfg5 (tools/ab_lev_refill.py).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "lev or cfg5 or exact_work or window or case_levels or pipeline or edge" \
  > gpurun_out/r5g_tests.log 2>&1 || { tail -40 gpurun_out/r5g_tests.log; exit 1; }
tail -2 gpurun_out/r5g_tests.log
timeout -k 10 300 python -u tools/ab_lev_refill.py 2 10 > gpurun_out/r5g_ab.log 2>&1 || { tail -20 gpurun_out/r5g_ab.log; exit 1; }
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 >> gpurun_out/r5g_ab.log 2>&1 || { tail -20 gpurun_out/r5g_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5g_ab.log
