#!/bin/bash
# Round 3 diagnostic: k_filter time with no left-row loads (timing only, wrong results) vs the real kernel.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_noleft.so
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_noleft -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
unset SPLINK_AMD_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_diagA2 -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
python - <<PY
import csv
for d in ("prof_diagA2", "prof_noleft"):
    for r in csv.DictReader(open(f"gpurun_out/{d}/run_kernel_stats.csv")):
        if "k_filter" in r["Name"]: print(d, "k_filter", float(r["AverageNs"]) / 1e3, "us")
PY
