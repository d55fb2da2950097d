#!/bin/bash
# Round 6: a kernel change -- parity subset (parity, windows, cfg2 and cfg5 columns at full size), then
# the default bench line (cfg2 + cfg5_columns) and its kernel statistics.  Usage: bash tools/gpu/r6c.sh TAG
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r6c}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_windows.py "tests/test_gpu_scale.py::test_cfg2_full_size" \
  "tests/test_gpu_scale.py::test_cfg5_columns_full_size" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['breakdown_ms']['gamma']); c=d['cfg5_columns']; print('cfg5', c['ms_per_step'], c['breakdown_ms'])
print(d['string_rates']['levenshtein_exact_pass'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 > gpurun_out/${TAG}_benchprof.json 2> gpurun_out/${TAG}_benchprof.err
echo "prof exit $?"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_cfg5 -o run -- python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > gpurun_out/${TAG}_benchprof_cfg5.json 2> gpurun_out/${TAG}_benchprof_cfg5.err
echo "prof exit $?"
