#!/bin/bash
# Counter passes of tools/ab_lev_refill.py (both Levenshtein exact kernels in one run), summarised per kernel.
# Usage: bash tools/gpu/pmc_lev.sh TAG [config]
TAG=${1:-lev}; CFG=${2:-2}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
pass() {
    local n=$1; shift
    timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmclev${n}_$TAG -o run -- \
        python -u tools/ab_lev_refill.py $CFG 2 > gpurun_out/pmclev${n}_$TAG.log 2>&1
}
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD || exit 1
pass 2 SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum || exit 1
python tools/pmc_summary.py gpurun_out/pmclev1_$TAG gpurun_out/pmclev2_$TAG --match "lev_refill|exact_simple" \
    --json gpurun_out/pmclev_$TAG.json
