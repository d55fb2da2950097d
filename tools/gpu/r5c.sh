#!/bin/bash
# Round 5: the whole GPU suite on the current tree, then the two-tier E+M A/B (abx/old.so = the round-5
# start's single-tier build), the rule-1 view-image A/B of the filter at cfg2, and the cfg5 bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_r5c.log 2>&1
rc=$?; echo "rc $rc" >> gpurun_out/t_r5c.log; tail -15 gpurun_out/t_r5c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu/ab_em.sh "abx/old.so" || exit 1
AB_MODES=1,21,1,21,11 timeout -k 10 200 python -u tools/ab_gamma.py > gpurun_out/ab_r5_views.log 2>&1
cat gpurun_out/ab_r5_views.log
