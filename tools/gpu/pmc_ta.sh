#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_r3b.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/tests_r3b.log; tail -4 gpurun_out/tests_r3b.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r3b.json 2> gpurun_out/bench_r3b.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bench_r3b.json')); b=d['breakdown_ms']
print('value %.4g ms/step %.4f' % (d['value'], d['ms_per_step']), {k: round(v, 4) for k, v in b.items()})
print('em', d['roofline_em']['avg_launch_ms'], d['roofline_em']['frac'], d['em_at_scale']['em_iteration'])"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --em-scale 0"
pass() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmcb${n} -o run -- $B > gpurun_out/pmcb${n}.log 2>&1; }
pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU || exit 1
pass 2 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum || exit 1
echo done
