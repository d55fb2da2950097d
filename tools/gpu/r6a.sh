#!/bin/bash
# Round 6, first box: GPU suite, the default bench line, the bench launcher at --gpus 2 (RCCL: must refuse on a
# one-GPU box; gloo: two ranks sharing the GPU, the N-rank bench path end to end).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6a_suite.log 2>&1 || { tail -30 gpurun_out/r6a_suite.log; exit 1; }
tail -1 gpurun_out/r6a_suite.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { tail -20 gpurun_out/r6a_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r6a_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['n_gpus'], d['ranks_seen'])"
timeout -k 10 120 python -u bench.py --gpus 2 > gpurun_out/r6a_bench2_nccl.json 2> gpurun_out/r6a_bench2_nccl.err
echo "--gpus 2 (nccl) exit $?"; tail -2 gpurun_out/r6a_bench2_nccl.err
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > gpurun_out/r6a_bench2_gloo.json 2> gpurun_out/r6a_bench2_gloo.err || { tail -20 gpurun_out/r6a_bench2_gloo.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r6a_bench2_gloo.json')); print(d['value'], d['ms_per_step'], d['n_gpus'], d['ranks_seen'], d['config']['candidate_pairs'])"
