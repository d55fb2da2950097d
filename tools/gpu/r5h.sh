#!/bin/bash
# Round 5: Levenshtein exact kernels -- parity subset, then tools/ab_lev_refill.py (refill vs per-lane in one
# process) with the in-tree library and the variants under splink_amd/abq/ (SPK_LEVQ_STEPS / SPK_LEVQ_ADOPT).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "lev or cfg5 or exact_work or window or case_levels or pipeline or edge" \
  > gpurun_out/r5h_tests.log 2>&1 || { tail -40 gpurun_out/r5h_tests.log; exit 1; }
tail -1 gpurun_out/r5h_tests.log
: > gpurun_out/r5h_ab.log
for lib in A ${LIBS:-abq/steps4.so abq/adopt8.so}; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  for cfg in 2 5; do
    echo "== $lib" >> gpurun_out/r5h_ab.log
    timeout -k 10 300 python -u tools/ab_lev_refill.py $cfg 6 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5h_ab.log || exit 1
  done
done
cat gpurun_out/r5h_ab.log
