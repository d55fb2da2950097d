#!/bin/bash
# Round 6: A/B of candidate libraries (splink_amd/base_*.so named in $1) against the in-tree one: parity subset per
# candidate, cfg2 bench lines alternating (two streams, one stream), one-stream kernel stats of each.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-"base_rg1.so base_rg2.so"}; TAG=${2:-r6u}
bash tools/gpu/ab_libs.sh "" "cfg2_full or levenshtein or simple_columns or pipeline" "$LIBS" > gpurun_out/${TAG}_tests.txt 2>&1 || { cat gpurun_out/${TAG}_tests.txt; exit 1; }
cat gpurun_out/${TAG}_tests.txt
for args in "--cfg5-steps 0" "--cfg5-steps 0 --gamma-streams 1"; do
  echo "== $args"
  BENCH_ARGS="$args" bash tools/gpu/ab_libs.sh "$LIBS" "" skip > gpurun_out/${TAG}_ab.txt 2>&1 || { cat gpurun_out/${TAG}_ab.txt; exit 1; }
  cat gpurun_out/${TAG}_ab.txt
done
for lib in A $LIBS; do
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
