#!/bin/bash
# Final record of the tree: smoke(), default bench line, rocprof kernel stats, the counter passes (pmc_record.sh),
# cfg5 bench (with its CPU baseline) + kernel stats.  Usage: record.sh TAG
TAG=${1:-rec}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
head -c 400 gpurun_out/bench_$TAG.json; echo
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cfg5-steps 0 > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || exit 1
bash tools/gpu/pmc_record.sh $TAG > gpurun_out/pmc_$TAG.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 --em-scale 0 > gpurun_out/bench_cfg5_$TAG.json 2> gpurun_out/bench_cfg5_$TAG.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_$TAG -o run -- python3 -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
python - <<PY
import json
for f in ("gpurun_out/bench_$TAG.json", "gpurun_out/bench_cfg5_$TAG.json"):
    d = json.load(open(f)); print(f, d["value"], d["ms_per_step"], d["breakdown_ms"]["gamma"], d["breakdown_ms"]["em_hist"])
PY
echo done
