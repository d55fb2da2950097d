#!/bin/bash
# Round 5: the 128-bit slow pass by lane refill (mode 1) against the per-lane kernel (mode 2) on the cells the
# character-bag compaction now hands it.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_lev_refill.py 5 6 2 1 2>&1 | grep -v amdgpu.ids > gpurun_out/r5ab_ab.log || { cat gpurun_out/r5ab_ab.log; exit 1; }
cat gpurun_out/r5ab_ab.log
