#!/bin/bash
# Round 3 diagnostic: k_filter time when its workgroups per CU are capped by padded LDS (3 and 2 waves per
# SIMD instead of 5): the room a concurrent exact pass would have.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in ab_occ3.so ab_occ2.so; do
  export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$lib -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
done
unset SPLINK_AMD_LIB
python - <<PY
import csv
for d in ("prof_ab_occ3.so", "prof_ab_occ2.so"):
    for r in csv.DictReader(open(f"gpurun_out/{d}/run_kernel_stats.csv")):
        if "k_filter" in r["Name"] or "exact_simple<true" in r["Name"]: print(d, r["Name"][:40], float(r["AverageNs"]) / 1e3, "us")
PY
