#!/bin/bash
# Kernel times per library build: rocprofv3 --kernel-trace --stats of a short bench run for the in-tree
# library (A) and each candidate (splink_amd/ab_*.so), top kernels printed per library.
# Usage: bash tools/gpu/prof_libs.sh "ab_x.so ab_y.so" [bench args]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}; ARGS=${2:-"--steps 5 --warmup 2 --no-cpu-baseline --em-scale 0"}
for lib in A $LIBS; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$lib -o run -- python -u bench.py $ARGS > gpurun_out/prof_$lib.json 2> gpurun_out/prof_$lib.err || exit 1
  python - <<PY
import csv, glob, json
d = json.load(open("gpurun_out/prof_$lib.json"))
print("== $lib", "ms/step %.4f" % d["ms_per_step"], "gamma %.4f" % d["breakdown_ms"]["gamma"])
f = glob.glob("gpurun_out/prof_$lib/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print(f"  {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
