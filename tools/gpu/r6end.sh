#!/bin/bash
# Round 6 end: the driver's own round-end steps on the final tree -- GPU suite, smoke(), default bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6end_suite.log 2>&1 || { tail -30 gpurun_out/r6end_suite.log; exit 1; }
tail -1 gpurun_out/r6end_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6end_smoke.log 2>&1 || { cat gpurun_out/r6end_smoke.log; exit 1; }
tail -1 gpurun_out/r6end_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6end_bench.json 2> gpurun_out/r6end_bench.err || { tail -20 gpurun_out/r6end_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r6end_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
