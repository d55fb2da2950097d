#!/bin/bash
# PMC passes over one short bench run (each pass its own process, hard time limit).
# Usage: bash scripts_gpu_pmc.sh TAG
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --em-scale 0 $BENCH_ARGS"
run_pass() {
    local n=$1; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc${n}_$TAG -o run \
        -- python -u bench.py $ARGS > gpurun_out/pmc${n}_$TAG.log 2>&1
}
run_pass 1 FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
run_pass 2 TCC_HIT_sum TCC_MISS_sum WRITE_SIZE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR || exit 1
run_pass 3 SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH || exit 1
echo done
