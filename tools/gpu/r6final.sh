#!/bin/bash
# Round 6 final records of the tree: kernel statistics (cfg2, cfg5), the counter passes and HBM traffic
# (pmc_record.sh), cfg5's Levenshtein counters, and the N-rank bench rehearsed with gloo on this one GPU.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6f -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cfg5-steps 0 > gpurun_out/benchprof_r6f.json 2> gpurun_out/benchprof_r6f.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_r6f -o run -- python3 -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 > gpurun_out/benchprof_cfg5_r6f.json 2> /dev/null || exit 1
bash tools/gpu/pmc_record.sh r6f > gpurun_out/pmc_r6f.txt 2>&1 || { tail -20 gpurun_out/pmc_r6f.txt; exit 1; }
bash tools/gpu/pmc_cfg5_lev.sh r6f > gpurun_out/pmclev_r6f_out.txt 2>&1 || { tail -20 gpurun_out/pmclev_r6f_out.txt; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 > gpurun_out/r6f_bench2_gloo.json 2> gpurun_out/r6f_bench2_gloo.err || { tail -20 gpurun_out/r6f_bench2_gloo.err; exit 1; }
head -c 300 gpurun_out/r6f_bench2_gloo.json; echo
echo done
