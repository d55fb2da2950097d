#!/bin/bash
# Round 5: kernel trace of the cfg5 100M-record share job: the E+M launches' own durations (first launch vs later).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/prof_fj_r5r -o run -- python3 -u tools/full_job.py --config 5 \
  --records 100000000 --surname-vocab 1000000 --chunks 64 --workers 16 --rules "$RULES" --shard 0/8 --no-parity \
  --out gpurun_out/fj100M_r5r.json > gpurun_out/fj100M_r5r.log 2>&1 || exit 1
f=$(ls gpurun_out/prof_fj_r5r/*/run_kernel_trace.csv gpurun_out/prof_fj_r5r/run_kernel_trace.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys, json
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_em' in r['Kernel_Name']]
for r in rows:
    print(r['Kernel_Name'][:60], round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, 4))
d = json.load(open('gpurun_out/fj100M_r5r.json'))
print('events em/iter', d['device_ms']['em_per_iter'])
PY
