# Round 3: UC at tighter PDHG tolerances under the new theta default (and a restart sweep at 1e-6)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
for e in 1e-7 1e-8 1e-9; do
  PHG_COOP=0 timeout -k 10 400 python3 -u tools/uc_iter_tail.py 64 10 $e > $O/uc_tail_$e.log 2>&1 || { echo "eps $e failed"; tail -3 $O/uc_tail_$e.log; exit 1; }
  echo "eps $e"; grep -E "Iter0|SUMMARY" $O/uc_tail_$e.log
done
i=0
for opts in '{"pdhg_beta_artificial": 0.5}' '{"pdhg_check_every": 64}' '{"pdhg_beta_sufficient": 0.1}' '{"pdhg_keep_omega": true}'; do
  i=$((i+1))
  UC_OPTS="$opts" PHG_COOP=0 timeout -k 10 300 python3 -u tools/uc_iter_tail.py 64 10 1e-6 > $O/uc_$i.log 2>&1 || { echo "run $i failed"; tail -3 $O/uc_$i.log; exit 1; }
  grep SUMMARY $O/uc_$i.log
done
PHG_COOP=0 timeout -k 10 300 python3 -u tools/uc_iter_tail.py 64 10 1e-6 > $O/uc_base.log 2>&1 && grep SUMMARY $O/uc_base.log
