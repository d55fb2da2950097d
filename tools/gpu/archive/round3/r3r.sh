#!/bin/bash
# Round 3: cfg5 kernel stats after the long-cell bins.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_r3r -o run -- python3 -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > gpurun_out/bench_cfg5_r3r.json 2> gpurun_out/bench_cfg5_r3r.err || exit 1
python - <<PY
import csv, json
d = json.load(open("gpurun_out/bench_cfg5_r3r.json"))
print(d["ms_per_step"], d["exact_cells_per_column"], d["string_rates"]["levenshtein_exact_pass"])
for r in list(csv.DictReader(open("gpurun_out/prof_cfg5_r3r/run_kernel_stats.csv")))[:14]: print(round(float(r["AverageNs"]) / 1e3, 1), "us x", r["Calls"], r["Name"][:70])
PY
echo done
