# Round 3: theta sweep, second pass (UC below 0.2; netdes / sslp 4096 / hydro around 0.5)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
i=0
for opts in '{"pdhg_primal_weight_theta": 0.05}' '{"pdhg_primal_weight_theta": 0.1, "pdhg_keep_omega": false}' '{"pdhg_primal_weight_theta": 0.1, "pdhg_beta_artificial": 0.5}' '{"pdhg_primal_weight_theta": 0.15}'; do
  i=$((i+1))
  UC_OPTS="$opts" PHG_COOP=0 timeout -k 10 300 python3 -u tools/uc_iter_tail.py 64 8 1e-6 > $O/uc_$i.log 2>&1 || { echo "run $i failed"; tail -3 $O/uc_$i.log; exit 1; }
  grep SUMMARY $O/uc_$i.log
done
for th in 0.8 0.6 0.5 0.4; do
  for c in "netdes" "sslp --scen 4096" "hydro"; do
    n=$(echo $c | cut -d' ' -f1)
    PHG_THETA=$th timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case $c > $O/${n}_$th.json 2> $O/${n}_$th.err || { tail -3 $O/${n}_$th.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$th.json')); r=d['roofline']; print('$n theta=$th', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'))"
  done
done
