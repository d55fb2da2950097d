#!/bin/bash
# Per-pass device times of the full-size job per library build (in-tree A and splink_amd/ab_*.so):
# tools/full_job.py without the parity sample.  Usage: bash tools/gpu/fulljob_ab.sh "ab_x.so" [full_job args]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}; ARGS=${2:-"--records 20000000 --shard 0/8 --iters 3"}
for lib in A $LIBS; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  timeout -k 10 500 python -u tools/full_job.py $ARGS --no-parity --out gpurun_out/fjab_$lib.json > gpurun_out/fjab_$lib.log 2>&1 || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/fjab_$lib.json')); print('$lib', d['pairs_this_gpu'], 'job %.2f s' % d['job_wall_s'], json.dumps(d['device_ms']))"
done
