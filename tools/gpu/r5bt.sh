#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bag_decisions or levenshtein_levels_exact or em_first_launch" \
  > gpurun_out/r5bt.log 2>&1 || { tail -40 gpurun_out/r5bt.log; exit 1; }
tail -1 gpurun_out/r5bt.log
