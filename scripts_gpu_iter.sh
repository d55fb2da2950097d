cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tests_r1s4.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r1s4.log; tail -15 gpurun_out/tests_r1s4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r1s4.json 2> gpurun_out/bench_r1s4.err || exit 1
cat gpurun_out/bench_r1s4.json
SPK_XCD_SWIZZLE=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r1s4_noswz.json 2> gpurun_out/bench_r1s4_noswz.err || exit 1
cat gpurun_out/bench_r1s4_noswz.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1s4 -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/benchprof_r1s4.json 2> gpurun_out/benchprof_r1s4.err || exit 1
echo done
