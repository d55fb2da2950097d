#!/bin/bash
# Round 3: the diagonal early exit pushed the Levenshtein exact kernel 4 VGPRs past its 96-VGPR cap (scratch
# spills, +108 MB of writes per call).  A/B: A = as committed; ab_v2 = diagonal only in the 128-bit scans
# (no spill); ab_lw4 = 4 waves per SIMD (no spill).  cfg2 / cfg5, then WRITE_SIZE of the three.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/ab_libs.sh "ab_v2.so ab_lw4.so" "cfg2_full or levenshtein or cfg5_address" || exit 1
bash tools/gpu/ab_cfg5.sh "ab_v2.so ab_lw4.so" || exit 1
for lib in A ab_v2.so; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw_$lib -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/pmcw_$lib.log 2>&1 || exit 1
done
unset SPLINK_AMD_LIB
python - <<PY
import csv, collections
for lib in ("A", "ab_v2.so"):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/pmcw_{lib}/run_counter_collection.csv")):
        if "exact_simple<true" in r["Kernel_Name"]: acc[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    print(lib, "exact<true> WRITE_SIZE KiB per dispatch", [round(sum(v)) for v in acc.values()][:6])
PY
echo done
