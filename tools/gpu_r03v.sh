# Round 3: primal-weight smoothing theta across the cases (PHG_THETA): UC tail sweep, then the
# farmer headline (time to conv), sslp, netdes and hydro benches at theta 0.8 (default) / 0.5 / 0.3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
i=0
for opts in '{"pdhg_primal_weight_theta": 0.2}' '{"pdhg_primal_weight_theta": 0.1}' '{"pdhg_primal_weight_theta": 0.3, "pdhg_beta_artificial": 0.5}' '{"pdhg_primal_weight_theta": 0.3, "pdhg_check_every": 64}'; do
  i=$((i+1))
  UC_OPTS="$opts" PHG_COOP=0 timeout -k 10 300 python3 -u tools/uc_iter_tail.py 64 8 1e-6 > $O/uc_$i.log 2>&1 || { echo "run $i failed"; tail -3 $O/uc_$i.log; exit 1; }
  grep SUMMARY $O/uc_$i.log
done
for th in 0.8 0.5 0.3; do
  PHG_THETA=$th timeout -k 10 200 python3 -u bench.py --conv-iters 20000 --cpu-seconds 0 > $O/farmer_$th.json 2> $O/farmer_$th.err || { tail -3 $O/farmer_$th.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/farmer_$th.json')); r=d['roofline']; t=d['time_to_conv']; print('farmer theta=$th', d['value'], d['ms_per_step'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'])"
  for c in sslp netdes hydro; do
    PHG_THETA=$th timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case $c > $O/${c}_$th.json 2> $O/${c}_$th.err || { tail -3 $O/${c}_$th.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${c}_$th.json')); r=d['roofline']; print('$c theta=$th', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'))"
  done
done
