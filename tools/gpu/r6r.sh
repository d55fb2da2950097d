#!/bin/bash
# Round 6: A/B of a library change (in-tree) against HEAD (splink_amd/base_ab.so): parity subset incl. the windows /
# split tests, then cfg2 (two streams, one stream) and cfg5 bench lines alternating, and a kernel trace of cfg2.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_windows.py \
  tests/test_gpu_parity.py tests/test_gpu_edge.py "tests/test_gpu_scale.py::test_cfg2_full_size" \
  > gpurun_out/r6r_tests.log 2>&1 || { tail -30 gpurun_out/r6r_tests.log; exit 1; }
tail -1 gpurun_out/r6r_tests.log
for args in "--cfg5-steps 0" "--cfg5-steps 0 --gamma-streams 1" "--config 5 --cfg5-steps 0"; do
  echo "== $args"
  BENCH_ARGS="$args" bash tools/gpu/ab_libs.sh "base_ab.so" "" skip > gpurun_out/r6r_ab.txt 2>&1 || { cat gpurun_out/r6r_ab.txt; exit 1; }
  cat gpurun_out/r6r_ab.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6r_prof -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 > /dev/null 2>&1 || exit 1
echo done
