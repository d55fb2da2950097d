#!/bin/bash
# One build -> measure round trip on the GPU box: parity tests (stop at a crash / timeout, plain failures
# continue), the default bench line, and a rocprofv3 kernel-trace summary of a short bench run.
# Usage: bash tools/gpu/iter.sh TAG [pytest -k expression]
TAG=${1:-it}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
if [ -n "$2" ]; then KOPT=(-k "$2"); else KOPT=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "${KOPT[@]}" > gpurun_out/tests_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_$TAG.log; tail -5 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python - <<PY
import json; d=json.load(open("gpurun_out/bench_$TAG.json")); b=d["breakdown_ms"]
print("value %.4g ms/step %.4f" % (d["value"], d["ms_per_step"]), {k: round(v, 4) for k, v in b.items()})
print("em", {k: d["roofline_em"][k] for k in ("avg_launch_ms", "frac")}, "headline", d["hbm_headline_contract"]["value"])
print("exact cells", d["exact_cells_per_column"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --em-scale 0 > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || exit 1
python - <<PY
import csv, glob
f = glob.glob("gpurun_out/prof_$TAG/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {r['Name'][:100]}")
PY
echo done
