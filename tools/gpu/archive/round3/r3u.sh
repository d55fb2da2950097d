#!/bin/bash
# Round 3: counter record of the cfg5 step (SQ issue / stall, TA / TCP) for the Levenshtein exact and slow passes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
B="python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0"
pass() { local n=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc${n}_cfg5 -o run -- $B > gpurun_out/pmc${n}_cfg5.log 2>&1; }
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU || exit 1
pass 2 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum || exit 1
pass 3 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
python tools/pmc_summary.py gpurun_out/pmc1_cfg5 gpurun_out/pmc2_cfg5 gpurun_out/pmc3_cfg5 --json gpurun_out/r3u_pmc_cfg5.json > gpurun_out/r3u_pmc_cfg5.txt 2>&1 || exit 1
grep -A12 "exact_simple<true\|slow_lev" gpurun_out/r3u_pmc_cfg5.txt | head -60
echo done
