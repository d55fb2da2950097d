#!/bin/bash
# One SQ counter pass per library build (instruction mix and wait share of the kernels matching REGEX).
# Usage: bash tools/gpu/pmc1_libs.sh "ab_x.so ..." [REGEX]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}; RX=${2:-k_filter}
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0"
for lib in A $LIBS; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -s KILL 200 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD} --kernel-trace --output-format csv -d gpurun_out/pmcq_$lib -o run -- $B > gpurun_out/pmcq_$lib.log 2>&1 || exit 1
  python - <<PY
import csv, glob, re, collections
v = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter(); dur = collections.defaultdict(float)
for f in glob.glob("gpurun_out/pmcq_$lib/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if not re.search("$RX", r["Kernel_Name"]): continue
        v[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            n[r["Kernel_Name"][:40]] += 1; dur[r["Kernel_Name"][:40]] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
for k, c in v.items():
    d = n[k]
    print("$lib", k, "disp", d, "us/disp %.1f" % (dur[k] / d / 1e3), " ".join(f"{x[8:]}={c[x]/d/1e6:.1f}M" for x in sorted(c)))
PY
done
