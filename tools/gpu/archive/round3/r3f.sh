#!/bin/bash
# Round 3: E+M launch split (fused vs histogram + finalize), default bench line, rocprof kernel stats and
# the counter record of the current tree.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u tools/ab_em.py > gpurun_out/ab_em_r3f.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ab_em.py 1000000 8 >> gpurun_out/ab_em_r3f.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_em_r3f.log
timeout -k 10 200 python -u bench.py > gpurun_out/bench_r3f.json 2> gpurun_out/bench_r3f.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3f -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/benchprof_r3f.json 2> gpurun_out/benchprof_r3f.err || exit 1
bash tools/gpu/r3_pmc.sh || exit 1
echo done
