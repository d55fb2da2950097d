#!/bin/bash
# Counter passes of the cfg5 comparison pass in its default mode (address: bag compaction, refill exact pass,
# 128-bit slow pass), summarised per kernel into gpurun_out/pmclev_TAG.json.  Usage: pmc_cfg5_lev.sh TAG
TAG=${1:-cfg5lev}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
pass() {
    local n=$1; shift
    timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmclev${n}_$TAG -o run -- \
        python -u tools/ab_lev_refill.py 5 2 2 > gpurun_out/pmclev${n}_$TAG.log 2>&1
}
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD || exit 1
pass 2 SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum || exit 1
python tools/pmc_summary.py gpurun_out/pmclev1_$TAG gpurun_out/pmclev2_$TAG --match "lev_refill|exact_simple|slow_lev|compact_lev|k_filter" \
    --json gpurun_out/pmclev_$TAG.json > gpurun_out/pmclev_$TAG.txt 2>&1 || exit 1
head -60 gpurun_out/pmclev_$TAG.txt
