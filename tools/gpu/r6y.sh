#!/bin/bash
# Round 6: tf sums from the direct (value, pattern) histogram -- tf GPU tests (edge, parity, cfg3 shares incl. the
# whole cfg3 on one GPU), then the whole cfg3 job record (r6v.sh) and its kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_gpu_edge.py \
  tests/test_gpu_parity.py "tests/test_gpu_scale.py::test_cfg3_shard_full_size" \
  "tests/test_gpu_scale.py::test_cfg3_one_gpu_full_size" -k "tf or link or cfg3" > gpurun_out/r6y_tests.log 2>&1 \
  || { tail -40 gpurun_out/r6y_tests.log; exit 1; }
tail -1 gpurun_out/r6y_tests.log
bash tools/gpu/r6v.sh > gpurun_out/r6y_fulljob.txt 2>&1 || { tail -20 gpurun_out/r6y_fulljob.txt; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r6_fulljob_cfg3_10Mx10M_1gpu.json')); print(d['wall_s'], d['job_wall_s'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6y_prof -o run -- python3 -u tools/full_job.py \
  --config 3 --records 10000000 --surname-vocab 300000 --shard 0/1 --chunks 16 --workers 16 --no-parity \
  --out gpurun_out/r6y_fulljob_cfg3_prof.json > gpurun_out/r6y_prof.log 2>&1 || { tail -30 gpurun_out/r6y_prof.log; exit 1; }
python3 - <<PY
import csv, glob, json
d = json.load(open("gpurun_out/r6y_fulljob_cfg3_prof.json")); print(d["wall_s"], d["job_wall_s"])
f = glob.glob("gpurun_out/r6y_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms total {float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>5}  {r['Name'][:80]}")
PY
