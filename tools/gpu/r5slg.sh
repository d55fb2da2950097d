#!/bin/bash
# Round 5: k_gamma_slow_lev grid (workgroups per CU: 8 in-tree, 3 / 6 in tools/abx), cfg5 γ pass, alternating.
# (the SPK_SLOWLEV_WG override was removed after this A/B: profiles/r5_ab_slow_grid.log)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/r5slg.log
for lib in A B C A B C; do
  case $lib in A) unset SPLINK_AMD_LIB;; B) export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/tools/abx/slow3.so;; C) export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/tools/abx/slow6.so;; esac
  echo "lib $lib" >> gpurun_out/r5slg.log
  timeout -k 10 200 python -u tools/ab_lev_refill.py 5 8 2 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5slg.log || exit 1
done
grep -E "^lib|kernel" gpurun_out/r5slg.log
