#!/bin/bash
# Round 6: cfg2 A/B of the email Levenshtein exact pass with the next cell's records and planes prefetched during
# the scan (in-tree, 3 waves/SIMD) against the in-tree build without it (ab_nopf.so, 4 waves/SIMD).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
BENCH_ARGS="--cfg5-steps 0" bash tools/gpu/ab_libs.sh "ab_nopf.so" > gpurun_out/r6j_ab.txt 2>&1 || { cat gpurun_out/r6j_ab.txt; exit 1; }
cat gpurun_out/r6j_ab.txt
for lib in A ab_nopf.so; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6j_prof_${lib//./_} -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 > /dev/null 2>&1 || exit 1
done
echo done
