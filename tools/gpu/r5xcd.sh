#!/bin/bash
# Round 5: XCD-grouped region mapping in k_filter (tools/abx/filter_xcd.so, -DSPK_FILTER_XCD=1) against the
# in-tree build, alternating, cfg2 and cfg5 γ pass; codes must match.
# (the SPK_FILTER_XCD variant was removed after this A/B: profiles/r5_ab_filter_xcd.log)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/r5xcd.log
for lib in A B A B; do
  if [ $lib == B ]; then export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/tools/abx/filter_xcd.so; else unset SPLINK_AMD_LIB; fi
  for c in 2 5; do
    echo "lib $lib cfg$c" >> gpurun_out/r5xcd.log
    timeout -k 10 200 python -u tools/ab_lev_refill.py $c 8 2 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5xcd.log || exit 1
  done
done
grep -E "^lib|kernel" gpurun_out/r5xcd.log
