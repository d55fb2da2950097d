#!/bin/bash
# Round 3: cfg5 columns bench + kernel stats; cfg4's per-GPU share full job (20M records, shard 0/8).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 > gpurun_out/bench_cfg5_r3l.json 2> gpurun_out/bench_cfg5_r3l.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bench_cfg5_r3l.json')); b=d['breakdown_ms']
print('cfg5', d['value'], d['ms_per_step'], 'gamma', b['gamma'], 'em', b['em_hist'], d['exact_cells_per_column'], d['string_rates']['levenshtein_exact_pass'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5_r3l -o run -- python3 -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
python - <<PY
import csv
for r in list(csv.DictReader(open("gpurun_out/prof_cfg5_r3l/run_kernel_stats.csv")))[:12]: print(round(float(r["AverageNs"]) / 1e3, 1), "us x", r["Calls"], r["Name"][:70])
PY
timeout -k 10 600 python -u tools/full_job.py --records 20000000 --shard 0/8 --out gpurun_out/fulljob_cfg4_r3l.json > gpurun_out/fulljob_cfg4_r3l.log 2>&1 || exit 1
python -c "
import json; d=json.load(open('gpurun_out/fulljob_cfg4_r3l.json')); print('cfg4', d['pairs_this_gpu'], d['job_wall_s'], d['device_ms'], d.get('parity_gamma'), d.get('parity_em'))"
echo done
