#!/bin/bash
# A/B of comparison-pass variants on cfg2 and on the cfg4 surname vocabulary.  Usage: bash scripts_gpu_ab2.sh TAG MODES
TAG=${1:-ab}; MODES=${2:-1,11,1,11}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_MODES=$MODES timeout -k 10 240 python -u tools/ab_gamma.py > gpurun_out/ab_$TAG.log 2>&1 || exit 1
AB_MODES=$MODES AB_VOCAB=300000 timeout -k 10 240 python -u tools/ab_gamma.py >> gpurun_out/ab_$TAG.log 2>&1 || exit 1
grep mode gpurun_out/ab_$TAG.log
