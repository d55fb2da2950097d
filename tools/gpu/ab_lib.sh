#!/bin/bash
# A/B of two builds on one box: the in-tree library (A) and splink_amd/ab_new.so (B), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ablib.log
for lib in A B A B; do
  if [ $lib == B ]; then export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_new.so; else unset SPLINK_AMD_LIB; fi
  echo "lib $lib" >> gpurun_out/ablib.log
  AB_MODES=${AB_MODES:-1} timeout -k 10 200 python -u tools/ab_gamma.py >> gpurun_out/ablib.log 2>&1 || exit 1
done
grep -E "^lib|mode" gpurun_out/ablib.log
