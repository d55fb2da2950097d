#!/bin/bash
# Bench line + full-job rows.  Usage: bash tools/gpu/fulljob_cfg4.sh TAG RECORDS SHARD
TAG=${1:-job}; REC=${2:-1000000}; SHARD=${3:-0/1}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$4" != "nobench" ]; then
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python - <<PY
import json; d=json.load(open("gpurun_out/bench_$TAG.json"))
print("value", d["value"], "ms/step", d["ms_per_step"]); print("breakdown", d["breakdown_ms"]); print("headline", d["hbm_headline_contract"]); print("roofline", d["roofline"]["frac"], d["roofline"]["algorithmic_bytes_per_launch"])
PY
fi
timeout -k 10 900 python -u tools/full_job.py --records $REC --shard $SHARD --out gpurun_out/fulljob_$TAG.json > gpurun_out/fulljob_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/fulljob_$TAG.log
exit $rc
