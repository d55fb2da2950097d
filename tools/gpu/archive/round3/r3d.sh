#!/bin/bash
# Round 3: EM parity subset with the write-through k_em_iter, A/B against the release-fence build, bench,
# rocprof kernel stats, and the counter record (r3_pmc.sh).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "em_ or cfg2_full or async or nccl or sharded or smoke or pipeline" > gpurun_out/tests_r3d.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3d.log; tail -2 gpurun_out/tests_r3d.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_score.sh "ab_pub0.so" || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r3d.json 2> gpurun_out/bench_r3d.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3d -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/benchprof_r3d.json 2> gpurun_out/benchprof_r3d.err || exit 1
bash tools/gpu/r3_pmc.sh || exit 1
echo done
