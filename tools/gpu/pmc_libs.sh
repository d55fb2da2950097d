#!/bin/bash
# SQ / LDS / TA counter passes of a short bench run per library build (A = in-tree, then candidates),
# summarised per kernel matching REGEX (tools/pmc_summary.py).
# Usage: bash tools/gpu/pmc_libs.sh "ab_x.so ..." [REGEX]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
LIBS=${1:-}; RX=${2:-k_filter}
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0"
for lib in A $LIBS; do
  if [ $lib == A ]; then unset SPLINK_AMD_LIB; else export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/$lib; fi
  pass() { local n=$1; shift; timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc${n}_$lib -o run -- $B > gpurun_out/pmc${n}_$lib.log 2>&1; }
  pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU || exit 1
  pass 2 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR || exit 1
  pass 3 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
  echo "== $lib"
  python tools/pmc_summary.py gpurun_out/pmc1_$lib gpurun_out/pmc2_$lib gpurun_out/pmc3_$lib --match "$RX" --json gpurun_out/pmc_$lib.json 2>&1 | head -30
done
