#!/bin/bash
# Round 6: where the tf stage of the whole cfg3 job on one GPU goes -- kernel trace of the full job (no parity).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6x_prof -o run -- python3 -u tools/full_job.py \
  --config 3 --records 10000000 --surname-vocab 300000 --shard 0/1 --chunks 16 --workers 16 --no-parity \
  --out gpurun_out/r6x_fulljob_cfg3.json > gpurun_out/r6x.log 2>&1 || { tail -30 gpurun_out/r6x.log; exit 1; }
python3 - <<PY
import csv, glob, json
d = json.load(open("gpurun_out/r6x_fulljob_cfg3.json")); print(d["wall_s"])
f = glob.glob("gpurun_out/r6x_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms total {float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>5}  {r['Name'][:80]}")
PY
