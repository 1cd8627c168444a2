# Round 3: theta above 0.8 on farmer (headline, with time to conv); sslp 4096 / hydro at 0.6-0.8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
for th in 1.0 0.9 0.8 0.7; do
  PHG_THETA=$th timeout -k 10 200 python3 -u bench.py --conv-iters 20000 --cpu-seconds 0 > $O/farmer_$th.json 2> $O/farmer_$th.err || { tail -3 $O/farmer_$th.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/farmer_$th.json')); r=d['roofline']; t=d['time_to_conv']; print('farmer theta=$th', d['value'], d['ms_per_step'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'])"
done
for th in 0.8 0.7 0.6 0.8 0.7 0.6; do
  for c in "sslp --scen 4096" "hydro"; do
    n=$(echo $c | cut -d' ' -f1)
    PHG_THETA=$th timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case $c > $O/${n}_$th.json 2> $O/${n}_$th.err || { tail -3 $O/${n}_$th.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$th.json')); r=d['roofline']; print('$n theta=$th', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'))"
  done
done
