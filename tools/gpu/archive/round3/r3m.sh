#!/bin/bash
# Round 3: A/B of the exact-pass grids (JW: 1/2/4 workgroups per CU per column; Levenshtein: 5/10 per CU).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/ab_libs.sh "ab_jw1.so ab_jw2.so ab_jw4.so ab_lev5.so ab_lev10.so" "cfg2_full" || exit 1
echo done
