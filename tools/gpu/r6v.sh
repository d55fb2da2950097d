#!/bin/bash
# Round 6: BASELINE configs[2] whole on one GPU -- cfg3 link_only 10M x 10M, tf on surname, 3.09e9 pairs in one
# context (ordinal windows), job wall and device memory by part.  No parity pass here: its host copies of every
# pair (gammas, rows, mp, the tf restatement) passed the box's 270 GiB host-memory cap; the parity at this size is
# tests/test_gpu_scale.py::test_cfg3_one_gpu_full_size (streamed, chunk by chunk).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/full_job.py --config 3 --records 10000000 --surname-vocab 300000 --shard 0/1 \
  --chunks 16 --workers 16 --no-parity --out gpurun_out/r6_fulljob_cfg3_10Mx10M_1gpu.json > gpurun_out/r6v_fulljob_cfg3.log 2>&1 \
  || { tail -30 gpurun_out/r6v_fulljob_cfg3.log; exit 1; }
tail -5 gpurun_out/r6v_fulljob_cfg3.log
head -c 3000 gpurun_out/r6_fulljob_cfg3_10Mx10M_1gpu.json
