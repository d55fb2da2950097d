#!/bin/bash
# Round-3 final record of the current tree: default bench line, rocprof kernel stats, the counter passes,
# cfg5 bench + kernel stats, and the practical HBM ceilings of plain streaming kernels.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r3s.json 2> gpurun_out/bench_r3s.err || exit 1
head -c 600 gpurun_out/bench_r3s.json; echo
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3s -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/benchprof_r3s.json 2> gpurun_out/benchprof_r3s.err || exit 1
bash tools/gpu/r3_pmc.sh > gpurun_out/pmc_r3s.txt 2>&1 || exit 1
timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 > gpurun_out/bench_cfg5_r3s.json 2> gpurun_out/bench_cfg5_r3s.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_r3s -o run -- python3 -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
timeout -k 10 200 python -u tools/hbm_ceiling.py > gpurun_out/hbm_ceiling_r3s.json 2> gpurun_out/hbm_ceiling_r3s.err || exit 1
cat gpurun_out/hbm_ceiling_r3s.json
echo done
