#!/bin/bash
# Round 6: A/B of the in-tree library against splink_amd/$1 (default base_sig0.so: the filter with runtime column
# counts only): parity subset, cfg2 (two streams, one stream) and cfg5 bench lines alternating, kernel stats of both.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B=${1:-base_sig0.so}; TAG=${2:-r6t}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_windows.py \
  tests/test_gpu_parity.py tests/test_gpu_edge.py "tests/test_gpu_scale.py::test_cfg2_full_size" \
  "tests/test_gpu_scale.py::test_cfg5_columns_full_size" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for args in "--cfg5-steps 0" "--cfg5-steps 0 --gamma-streams 1" "--config 5 --cfg5-steps 0"; do
  echo "== $args"
  BENCH_ARGS="$args" bash tools/gpu/ab_libs.sh "$B" "" skip > gpurun_out/${TAG}_ab.txt 2>&1 || { cat gpurun_out/${TAG}_ab.txt; exit 1; }
  cat gpurun_out/${TAG}_ab.txt
done
for lib in A $B; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_${lib%.so} -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 --gamma-streams 1 > /dev/null 2>&1 || exit 1
done
unset SPLINK_AMD_LIB
python3 - <<PY
import csv, glob
for d in sorted(glob.glob("gpurun_out/${TAG}_prof_*")):
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
    for r in list(csv.DictReader(open(f)))[:4]:
        print(d[-12:], f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {r['Name'][:70]}")
PY
