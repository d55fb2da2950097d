#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/tests_r3c.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3c.log; tail -6 gpurun_out/tests_r3c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_rules.py > gpurun_out/ab_rules.log 2>&1 || exit 1
grep pairs gpurun_out/ab_rules.log
timeout -k 10 240 python -u tools/ab_em.py > gpurun_out/ab_em.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/ab_em.log
