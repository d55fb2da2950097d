#!/bin/bash
# Round 5: full GPU suite, the Levenshtein kernel A/B at cfg2 / cfg5, then the cfg2 / cfg5 bench lines with
# kernel statistics (tools/gpu/r5d.sh).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5k_suite.log 2>&1 || { tail -30 gpurun_out/r5k_suite.log; exit 1; }
tail -1 gpurun_out/r5k_suite.log
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 0 1 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r5k_ab.log || exit 1
timeout -k 10 300 python -u tools/ab_lev_refill.py 2 8 0 2 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5k_ab.log || exit 1
cat gpurun_out/r5k_ab.log
bash tools/gpu/r5d.sh r5k
