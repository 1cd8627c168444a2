# round 6 end: every BASELINE config's bench line with the final code (conv legs included)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_secondary; mkdir -p $O
run() {  # tag, bench args...
  tag=$1; shift
  timeout -k 10 400 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d.get('time_to_conv',{}); r=d['roofline']
print('$tag', d['config'].get('pdhg_layout'), d['value'], d['ms_per_step'], r.get('frac'), t.get('seconds'), t.get('ph_iters'), t.get('conv'))"
}
run sslp_4096 --case sslp --scen 4096 --conv-time 60
run netdes_1024 --case netdes
run hydro_2000 --case hydro
run hydro_20000 --case hydro --scen 20000
run uc_64 --case uc --steps 3 --warmup 1 --conv-iters 0
