#!/bin/bash
# Round 5: two-phase Levenshtein passes -- parity subset, then tools/ab_lev_refill.py over cap variants.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "lev or cfg5 or exact_work or window or case_levels or pipeline or edge or strings_past" \
  > gpurun_out/r5i_tests.log 2>&1 || { tail -40 gpurun_out/r5i_tests.log; exit 1; }
tail -1 gpurun_out/r5i_tests.log
timeout -k 10 400 python -u tools/ab_lev_refill.py 5 6 0:0:0 0:0:8 0:0:12 0:0:16 0:16:8 0:24:8 0:32:8 1:0:8 \
  2>&1 | grep -v amdgpu.ids > gpurun_out/r5i_ab5.log || { tail gpurun_out/r5i_ab5.log; exit 1; }
cat gpurun_out/r5i_ab5.log
timeout -k 10 300 python -u tools/ab_lev_refill.py 2 8 0:0:0 1:0:0 2>&1 | grep -v amdgpu.ids > gpurun_out/r5i_ab2.log || exit 1
cat gpurun_out/r5i_ab2.log
