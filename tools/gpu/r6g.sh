#!/bin/bash
# Round 6: A/B of the Levenshtein exact pass with LDS threshold tables (in-tree) against the previous build
# (splink_amd/ab_base.so), kernel stats of both, then the cfg5 address-pass counters.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/ab_libs.sh "ab_base.so" > gpurun_out/r6g_ab.txt 2>&1 || { cat gpurun_out/r6g_ab.txt; exit 1; }
cat gpurun_out/r6g_ab.txt
for lib in A ab_base.so; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6g_prof_${lib//./_} -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cfg5-steps 0 > /dev/null 2>&1 || exit 1
done
unset SPLINK_AMD_LIB
bash tools/gpu/pmc_cfg5_lev.sh r6 > gpurun_out/pmclev_r6_out.txt 2>&1 || exit 1
echo done
