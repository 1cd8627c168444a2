# round 6: UC 64 with the cost-based rho -- eps schedules that hold the loose tolerances longer
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_uc3; mkdir -p $O
for X in "1e-3:1e-5,1.2e-4:1e-6,0:1e-7" "3e-3:1e-5,1.2e-4:2e-6,0:1e-7"; do
  tag=$(echo $X | tr ':,' '__')
  timeout -k 10 420 python -u bench.py --case uc --uc-rho cost --steps 3 --warmup 1 --cpu-seconds 0 --conv-time 120 --eps-schedule $X > $O/uc_$tag.json 2> $O/uc_$tag.err || { tail -5 $O/uc_$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/uc_$tag.json').read().strip().splitlines()[-1]); t=d['time_to_conv']
print('uc $X', t['seconds'], t['ph_iters'], t['conv'], t.get('converged'), t.get('final_pdhg_eps'), t.get('Eobj'))"
done
