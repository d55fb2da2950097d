#!/bin/bash
# Round 6 final tree: the tf / edge GPU tests, then the records of r6final.sh (kernel statistics, counters, traffic,
# cfg5 Levenshtein counters, the 2-rank gloo rehearsal).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py \
  > gpurun_out/r6z_tests.log 2>&1 || { tail -30 gpurun_out/r6z_tests.log; exit 1; }
tail -1 gpurun_out/r6z_tests.log
bash tools/gpu/r6final.sh
