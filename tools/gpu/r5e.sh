#!/bin/bash
# Round 5: E+M A/B (two tiers + uncounted top pattern vs abx/old.so, the round-4 kernel) at the tiled cfg2 /
# cfg5 sizes and at the real cfg5 100M-record share (no parity), the prefetch A/B of that job's wall, then
# the cfg2 / cfg5 bench lines with kernel statistics (tools/gpu/r5d.sh).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu/ab_em.sh "abx/old.so" || exit 1
RULES="l.surname = r.surname|l.dob = r.dob and l.city = r.city"
for run in A_pre A_nopre old_nopre; do
  case $run in
    A_pre) unset SPLINK_AMD_LIB; X="";;
    A_nopre) unset SPLINK_AMD_LIB; X="--no-prefetch";;
    old_nopre) export SPLINK_AMD_LIB=$GRAFT_REPO_ROOT/splink_amd/abx/old.so; X="--no-prefetch";;
  esac
  timeout -k 10 400 python -u tools/full_job.py --config 5 --records 100000000 --surname-vocab 1000000 --chunks 64 \
    --workers 16 --rules "$RULES" --shard 0/8 --no-parity $X --out gpurun_out/fj100M_r5_$run.json \
    > gpurun_out/fj100M_r5_$run.log 2>&1 || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/fj100M_r5_$run.json'))
print('$run', 'wall', round(d['job_wall_s'],3), 'em/iter', round(d['device_ms']['em_per_iter_mean'],4), 'gamma', round(d['device_ms']['gamma_pass'],2), {k: round(v,3) for k,v in d['wall_s'].items()}, {k: round(v,3) for k,v in d['job_timings_s'].items()})"
done
unset SPLINK_AMD_LIB
bash tools/gpu/r5d.sh r5e
