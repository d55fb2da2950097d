#!/bin/bash
# Round 3: filter-signature A/B (parity subset + alternating bench), then the per-rule pass split.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/ab_libs.sh "ab_sig3w5.so ab_sig2w6.so ab_sig4w4.so ab_sig2w8.so" "cfg2_full or simple_columns or case_levels or pipeline" || exit 1
timeout -k 10 300 python -u tools/ab_rules.py > gpurun_out/ab_rules.log 2>&1 || exit 1
cat gpurun_out/ab_rules.log
