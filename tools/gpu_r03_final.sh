# Round 3 final: the headline round profile (kernel trace + FETCH / WRITE PMC passes + the full
# default bench line), then the secondary configs' bench lines with time to conv
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_profile.sh > gpurun_out/round_profile.log 2>&1
rc=$?; echo "round profile exit $rc"; tail -2 gpurun_out/round_profile.log | cut -c1-400
[ $rc -eq 0 ] || exit 1
O=gpurun_out/r03final
mkdir -p $O
for c in "sslp --scen 2048" "netdes --scen 1024" "hydro" "uc"; do
  n=$(echo $c | cut -d' ' -f1)
  PHG_COOP=0 timeout -k 10 400 python3 -u bench.py --case $c --conv-time 60 --cpu-seconds 0 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -3 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; t=d['time_to_conv']; print('$n', d['value'], d['ms_per_step'], r.get('frac'), r.get('pdhg_iters_per_scen_per_step'), t.get('seconds'), t.get('ph_iters'), t.get('conv'), t.get('converged'))"
done
