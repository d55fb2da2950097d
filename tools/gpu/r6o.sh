#!/bin/bash
# Round 6: A/B of a filter change (in-tree) against HEAD before it (splink_amd/base_ab.so): parity subset incl. the
# windows / view-launch / split tests, cfg2 and cfg5 bench alternating, kernel traces of cfg2 (one stream).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_windows.py \
  tests/test_gpu_parity.py "tests/test_gpu_scale.py::test_cfg2_full_size" "tests/test_gpu_scale.py::test_cfg5_columns_full_size" \
  > gpurun_out/r6o_tests.log 2>&1 || { tail -30 gpurun_out/r6o_tests.log; exit 1; }
tail -1 gpurun_out/r6o_tests.log
BENCH_ARGS="--cfg5-steps 0" bash tools/gpu/ab_libs.sh "base_ab.so" "" skip > gpurun_out/r6o_ab.txt 2>&1 || { cat gpurun_out/r6o_ab.txt; exit 1; }
cat gpurun_out/r6o_ab.txt
BENCH_ARGS="--config 5 --cfg5-steps 0" bash tools/gpu/ab_libs.sh "base_ab.so" "" skip > gpurun_out/r6o_ab5.txt 2>&1 || { cat gpurun_out/r6o_ab5.txt; exit 1; }
cat gpurun_out/r6o_ab5.txt
for lib in A base_ab.so; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6o_prof_${lib//./_} -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 --gamma-streams 1 > /dev/null 2>&1 || exit 1
done
echo done
