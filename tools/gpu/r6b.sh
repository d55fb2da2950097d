#!/bin/bash
# Round 6: the cfg3 one-GPU test (3.09e9 link_only pairs + tf), the windows / prefetch / derived tests, and the
# default bench line with its cfg5_columns sub-record.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=0 \
  tests/test_gpu_windows.py tests/test_gpu_derived.py "tests/test_gpu_scale.py::test_cfg3_shard_full_size" \
  "tests/test_gpu_scale.py::test_cfg3_one_gpu_full_size" -m gpu > gpurun_out/r6b_tests.log 2>&1 || { tail -40 gpurun_out/r6b_tests.log; exit 1; }
grep -E "passed|failed|s call" gpurun_out/r6b_tests.log | tail -15
timeout -k 10 300 python -u bench.py > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err || { tail -20 gpurun_out/r6b_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r6b_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d['cfg5_columns'])[:1500])"
