#!/bin/bash
# Parity subset on the candidate library (ab_new.so), then the two-library timing A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_new.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "${K:-levenshtein or jaro or udf or case_levels or scale or pipeline or simple_columns or strings or lists or implied}" > gpurun_out/tests_abnew.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/tests_abnew.log; tail -2 gpurun_out/tests_abnew.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts_gpu_ablib.sh
