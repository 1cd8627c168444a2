# round 6: which of the block<=256 defaults (check 96, beta_art 0.15) fails on held-out sslp_5_25_50
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_d; mkdir -p $O
run() {  # tag, bench args...
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d['time_to_conv']; r=d['roofline']
print('$tag', d['config']['pdhg_layout'], d['config'].get('lanes_per_scenario'), d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), r.get('max_pdhg_iters'), t['seconds'], t['ph_iters'], t['conv'])"
}
run sslp5_c96 --case sslp --instance sslp_5_25_50 --conv-time 60 --check-every 96 --beta-art 0.25
run sslp5_b15 --case sslp --instance sslp_5_25_50 --conv-time 60 --check-every 64 --beta-art 0.15
run sslp15_default --case sslp --conv-time 60
run sslp15_base --case sslp --conv-time 60 --check-every 64 --beta-art 0.25
