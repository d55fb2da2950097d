#!/bin/bash
# cfg5 columns (free-text address Levenshtein-4) at cfg2 size: bench line + kernel trace.  Usage: bash scripts_gpu_cfg5.sh TAG
TAG=${1:-c5}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 --em-scale 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || exit 1
echo done
