#!/bin/bash
# Counter passes of the bench command (end of round 2; the FETCH_SIZE calibration is in profiles/r2_calib_fetch_*).
# Usage: bash tools/gpu/pmc.sh TAG
TAG=${1:-pmc}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 8"
pass() {
    local n=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc${n}_$TAG -o run -- $B > gpurun_out/pmc${n}_$TAG.log 2>&1
}
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU || exit 1
pass 2 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum || exit 1
pass 3 FETCH_SIZE || exit 1
pass 4 WRITE_SIZE || exit 1
echo done
