#!/bin/bash
# Round 6: device-resident tf results -- the tf GPU tests, then the whole cfg3 job on one GPU (r6v.sh).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_edge.py \
  tests/test_gpu_parity.py -k "tf or link" > gpurun_out/r6w_tests.log 2>&1 || { tail -30 gpurun_out/r6w_tests.log; exit 1; }
tail -1 gpurun_out/r6w_tests.log
bash tools/gpu/r6v.sh
