#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_MODES=${AB_MODES:-1,1001,3,1,1001} timeout -k 10 300 python -u tools/ab_gamma.py > gpurun_out/ab3.log 2>&1 || exit 1
grep mode gpurun_out/ab3.log
