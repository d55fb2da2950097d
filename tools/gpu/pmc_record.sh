#!/bin/bash
# Counter record of the bench command: SQ issue / stall, LDS, TA / TCP, then FETCH_SIZE and WRITE_SIZE in their
# own passes; summarised into gpurun_out/TAG_pmc_kernels.json and TAG_traffic.json.  Usage: pmc_record.sh TAG
TAG=${1:-rec}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 8 --cfg5-steps 0"
pass() { local n=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc${n}_$TAG -o run -- $B > gpurun_out/pmc${n}_$TAG.log 2>&1; }
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU || exit 1
pass 2 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum || exit 1
pass 3 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass 4 FETCH_SIZE || exit 1
pass 5 WRITE_SIZE || exit 1
python tools/pmc_summary.py gpurun_out/pmc1_$TAG gpurun_out/pmc2_$TAG gpurun_out/pmc3_$TAG --json gpurun_out/${TAG}_pmc_kernels.json > gpurun_out/${TAG}_pmc_summary.txt 2>&1 || exit 1
python tools/traffic.py --fetch gpurun_out/pmc4_$TAG --write gpurun_out/pmc5_$TAG --out gpurun_out/${TAG}_traffic.json > /dev/null || exit 1
head -40 gpurun_out/${TAG}_pmc_summary.txt
