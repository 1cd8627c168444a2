# round 6 shard table: farmer cm=10 per-GPU shard sizes, 2 runs each, bench defaults, no conv leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_shard2; mkdir -p $O
for rep in 1 2; do
  for sc in 10000 5000 2500 1250; do
    timeout -k 10 300 python -u bench.py --cpu-seconds 0 --conv-iters 0 --scen $sc > $O/s${sc}_$rep.json 2> $O/s${sc}_$rep.err || { tail -5 $O/s${sc}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/s${sc}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$sc', '$rep', d['ms_per_step'], r.get('avg_launch_ms'), d.get('host_and_exchange_ms_per_step'), d['value'], r.get('frac'))"
  done
done
