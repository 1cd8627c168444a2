# UC 64 with the reference's cost-based rho: fixed eps 1e-7 vs the conv-keyed eps schedule
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_uc; mkdir -p $O
for tag in sched fixed; do
  if [ $tag = sched ]; then X="--eps-schedule 1e-2:1e-5,1e-3:1e-6,0:1e-7"; else X=""; fi
  timeout -k 10 420 python -u bench.py --case uc --uc-rho cost --steps 3 --warmup 1 --cpu-seconds 0 --conv-time 120 $X > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d['time_to_conv']
print('$tag', d['ms_per_step'], t['seconds'], t['ph_iters'], t['conv'], t.get('seconds_iter0_and_first_20_ph_iters'), t.get('final_pdhg_eps'), t.get('Eobj'))"
done
