#!/bin/bash
# Round 6: two-stream split of the comparison pass -- its tests, the parity subset, then bench with 1 and 2 streams
# alternating (cfg2 and cfg5) and a kernel trace of each.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_windows.py \
  tests/test_gpu_parity.py "tests/test_gpu_scale.py::test_cfg2_full_size" "tests/test_gpu_scale.py::test_cfg5_columns_full_size" \
  > gpurun_out/r6k_tests.log 2>&1 || { tail -40 gpurun_out/r6k_tests.log; exit 1; }
tail -1 gpurun_out/r6k_tests.log
: > gpurun_out/r6k_ab.log
for rep in 1 2; do
  for s in 2 1; do
    for cfg in 2 5; do
      timeout -k 10 200 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 --gamma-streams $s > gpurun_out/r6k_b${cfg}_$s.json 2>/dev/null || exit 1
      python -c "
import json; d=json.load(open('gpurun_out/r6k_b${cfg}_$s.json')); b=d['breakdown_ms']
print('cfg$cfg streams $s', 'ms/step %.4f' % d['ms_per_step'], 'gamma %.4f' % b['gamma'], 'em %.4f' % (b['em_hist'] + b['em_final']))" >> gpurun_out/r6k_ab.log
    done
  done
done
cat gpurun_out/r6k_ab.log
for s in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6k_prof_$s -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --em-scale 0 --cfg5-steps 0 --gamma-streams $s > /dev/null 2>&1 || exit 1
done
echo done
