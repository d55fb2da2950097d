#!/bin/bash
# Round 3: GPU tests (slow-list launch skipping), E+M stage stamps.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_r3g.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3g.log; tail -2 gpurun_out/tests_r3g.log
[ $rc -ne 0 ] && exit $rc
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_stamps.so timeout -k 10 200 python -u tools/ab_em_stamps.py > gpurun_out/em_stamps.log 2>&1 || exit 1
SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_stamps.so timeout -k 10 200 python -u tools/ab_em_stamps.py 1000000 8 >> gpurun_out/em_stamps.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/em_stamps.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --em-scale 0 > gpurun_out/bench_r3g.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_r3g.json')); print(d['ms_per_step'], d['breakdown_ms']['gamma'], d['breakdown_ms']['em_hist'])"
echo done
export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/ab_diagleft.so
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_diagleft -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
unset SPLINK_AMD_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_diagA -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --em-scale 0 > /dev/null 2>&1 || exit 1
python - <<PY
import csv
for d in ("prof_diagA", "prof_diagleft"):
    for r in csv.DictReader(open(f"gpurun_out/{d}/run_kernel_stats.csv")):
        if "k_filter" in r["Name"]: print(d, "k_filter", float(r["AverageNs"]) / 1e3, "us")
PY
