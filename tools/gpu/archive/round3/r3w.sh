#!/bin/bash
# Round 3: filter regions per CU (10 / 40 vs 20) and a fire-and-forget atomic code add in the Levenshtein exact
# pass -- cfg2 and cfg5 A/B against the tree.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/ab_libs.sh "ab_reg10.so ab_reg40.so ab_xatomic.so" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_xatomic.so" || exit 1
echo done
