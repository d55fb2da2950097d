#!/bin/bash
# Round 5: diagonal exits in every scan phase + two-phase caps; A (LEV_WAVES 5) vs abq/w4.so (LEV_WAVES 4).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_windows.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "lev or cfg5 or exact_work or window or case_levels or pipeline or edge or strings_past or udf" \
  > gpurun_out/r5j_tests.log 2>&1 || { tail -40 gpurun_out/r5j_tests.log; exit 1; }
tail -1 gpurun_out/r5j_tests.log
: > gpurun_out/r5j_ab.log
for lib in A abq/w4.so; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  echo "== $lib" >> gpurun_out/r5j_ab.log
  timeout -k 10 400 python -u tools/ab_lev_refill.py 5 6 0:0:0 0:0:8 0:0:16 0:16:8 0:24:12 0:32:16 1:0:0 \
    2>&1 | grep -v amdgpu.ids >> gpurun_out/r5j_ab.log || exit 1
  timeout -k 10 300 python -u tools/ab_lev_refill.py 2 8 0:0:0 1:0:0 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5j_ab.log || exit 1
done
cat gpurun_out/r5j_ab.log
