# round 6: held-out A/B of the per-layout defaults, then the VALU class mix
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_c; mkdir -p $O
run() {  # tag, bench args...
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 --conv-time 120 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d['time_to_conv']; r=d['roofline']
print('$tag', d['config']['pdhg_layout'], d['config'].get('lanes_per_scenario'), d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), r.get('max_pdhg_iters'), t['seconds'], t['ph_iters'], t['conv'])"
}
run sslp5_default --case sslp --instance sslp_5_25_50
run sslp5_base --case sslp --instance sslp_5_25_50 --check-every 64 --beta-art 0.25
run net10_default --case netdes --instance network-10-20-H-01
run net10_base --case netdes --instance network-10-20-H-01 --check-every 64 --beta-art 0.25
run net10_c32 --case netdes --instance network-10-20-H-01 --check-every 32
