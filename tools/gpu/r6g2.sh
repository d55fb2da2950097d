#!/bin/bash
# Round 6: on the one-GPU box, bench.py --gpus 2 (RCCL) must refuse with a clear message and a non-zero exit.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r6g2_bench.out 2> gpurun_out/r6g2_bench.err
rc=$?
echo "bench.py --gpus 2 exit $rc" | tee gpurun_out/r6_bench_gpus2_one_gpu_box.log
tail -3 gpurun_out/r6g2_bench.err | tee -a gpurun_out/r6_bench_gpus2_one_gpu_box.log
echo "stdout bytes: $(wc -c < gpurun_out/r6g2_bench.out)" | tee -a gpurun_out/r6_bench_gpus2_one_gpu_box.log
