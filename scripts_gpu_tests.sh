#!/bin/bash
# GPU parity tests only (verbose, per-test durations).  Usage: bash scripts_gpu_tests.sh TAG [pytest args]
TAG=${1:-run}
shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --durations=15 --timeout 300 --timeout-method thread "$@" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_$TAG.log
tail -25 gpurun_out/tests_$TAG.log
exit $rc
