# round 6: held-out A/B of keep_omega (blend default vs fresh), sslp at 60 s conv legs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_e; mkdir -p $O
run() {  # tag, bench args...
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d['time_to_conv']; r=d['roofline']
print('$tag', d['config']['pdhg_layout'], d['config'].get('lanes_per_scenario'), d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), r.get('max_pdhg_iters'), t['seconds'], t['ph_iters'], t['conv'])"
}
run sslp5_default --case sslp --instance sslp_5_25_50 --conv-time 60
run sslp5_fresh --case sslp --instance sslp_5_25_50 --conv-time 60 --keep-omega fresh
run net10_default --case netdes --instance network-10-20-H-01
run net10_fresh --case netdes --instance network-10-20-H-01 --keep-omega fresh
