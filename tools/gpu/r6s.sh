#!/bin/bash
# Round 6: graph replay of the comparison pass -- tests (windows / split / graph, parity, edge, cfg2 and cfg5 columns at
# full size), then bench lines with and without the graph alternating (cfg2 split, cfg2 one stream, cfg5), a trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_windows.py \
  tests/test_gpu_parity.py tests/test_gpu_edge.py "tests/test_gpu_scale.py::test_cfg2_full_size" \
  "tests/test_gpu_scale.py::test_cfg5_columns_full_size" > gpurun_out/r6s_tests.log 2>&1 || { tail -30 gpurun_out/r6s_tests.log; exit 1; }
tail -1 gpurun_out/r6s_tests.log
: > gpurun_out/r6s_ab.log
for rep in 1 2; do
  for args in "" "--gamma-streams 1" "--config 5"; do
    for g in "" "--no-gamma-graph"; do
      timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 $args $g > gpurun_out/r6s_b.json 2>/dev/null || exit 1
      python -c "
import json; d=json.load(open('gpurun_out/r6s_b.json')); b=d['breakdown_ms']
print('[$args] [$g]', 'ms/step %.4f' % d['ms_per_step'], 'gamma %.4f' % b['gamma'], 'em %.4f' % (b['em_hist'] + b['em_final']), 'host gammas call %.3f' % b['host_wall_gammas_call'])" >> gpurun_out/r6s_ab.log
    done
  done
done
cat gpurun_out/r6s_ab.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6s_prof -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 > /dev/null 2>&1 || exit 1
echo done
