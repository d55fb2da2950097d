#!/bin/bash
# Round 6: cfg5 A/B of the banded 65-128-unit Levenshtein scan (in-tree) against HEAD before it (ab_base.so) and
# the in-tree build without the band (ab_noband.so: only the np <= 7 / np = 8 split of k_gamma_slow_lev).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
BENCH_ARGS="--config 5" bash tools/gpu/ab_libs.sh "ab_base.so ab_noband.so" "levenshtein or case_levels or cfg5 or slow" > gpurun_out/r6i_ab.txt 2>&1 || { cat gpurun_out/r6i_ab.txt; exit 1; }
cat gpurun_out/r6i_ab.txt
for lib in A ab_base.so; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6i_prof_${lib//./_} -o run -- python3 -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
done
echo done
