# Round 3: UC restart / primal-weight sweep (PH iterations 1..8 at S = 64, eps 1e-6)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
i=0
for opts in '{}' '{"pdhg_primal_weight_theta": 0.5}' '{"pdhg_primal_weight_theta": 0.3}' '{"pdhg_keep_omega": true}' '{"pdhg_keep_omega": false}' '{"pdhg_beta_artificial": 0.36}' '{"pdhg_beta_artificial": 0.5}' '{"pdhg_beta_sufficient": 0.4}' '{"pdhg_check_every": 64}' '{}'; do
  i=$((i+1))
  UC_OPTS="$opts" PHG_COOP=0 timeout -k 10 300 python3 -u tools/uc_iter_tail.py 64 8 1e-6 > $O/uc_$i.log 2>&1 || { echo "run $i failed"; tail -3 $O/uc_$i.log; exit 1; }
  grep SUMMARY $O/uc_$i.log
done
