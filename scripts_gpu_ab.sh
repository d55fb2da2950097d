#!/bin/bash
# A/B timing of the comparison-pass variants + PMC passes over the same script.  Usage: bash scripts_gpu_ab.sh TAG
TAG=${1:-ab}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/ab_gamma.py > gpurun_out/ab_$TAG.log 2>&1 || exit 1
pass() {
    local n=$1; shift
    timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/abpmc${n}_$TAG -o run \
        -- python -u tools/ab_gamma.py > gpurun_out/abpmc${n}_$TAG.log 2>&1
}
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU || exit 1
pass 2 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum || exit 1
echo done
