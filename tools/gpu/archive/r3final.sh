#!/bin/bash
# Round-3 final record of the tree: smoke(), default bench line, rocprof kernel stats, the counter passes,
# cfg5 bench + kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r3final.log 2>&1 || exit 1
tail -1 gpurun_out/smoke_r3final.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r3final.json 2> gpurun_out/bench_r3final.err || exit 1
head -c 400 gpurun_out/bench_r3final.json; echo
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3final -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/benchprof_r3final.json 2> gpurun_out/benchprof_r3final.err || exit 1
bash tools/gpu/r3_pmc.sh > gpurun_out/pmc_r3final.txt 2>&1 || exit 1
timeout -k 10 240 python -u bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline --em-scale 0 > gpurun_out/bench_cfg5_r3final.json 2> gpurun_out/bench_cfg5_r3final.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_r3final -o run -- python3 -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
python - <<PY
import json
for f in ("gpurun_out/bench_r3final.json", "gpurun_out/bench_cfg5_r3final.json"):
    d = json.load(open(f)); print(f, d["value"], d["ms_per_step"], d["breakdown_ms"]["gamma"], d["breakdown_ms"]["em_hist"])
PY
echo done
