#!/bin/bash
# Round 5: regrouping by predicted trip count (lev_trip_bin) in the per-lane exact pass and the slow pass --
# Levenshtein parity subset, then the kernel A/B at cfg5 / cfg2.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "lev or cfg5 or exact_work or window or case_levels or pipeline or edge or strings_past or udf" \
  > gpurun_out/r5n_tests.log 2>&1 || { tail -40 gpurun_out/r5n_tests.log; exit 1; }
tail -1 gpurun_out/r5n_tests.log
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 0 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r5n_ab.log || { cat gpurun_out/r5n_ab.log; exit 1; }
timeout -k 10 300 python -u tools/ab_lev_refill.py 2 8 0 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5n_ab.log || exit 1
cat gpurun_out/r5n_ab.log
