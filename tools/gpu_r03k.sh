# Round 3: the folded PH update at S*N = 1e8 (1e6 x 100) under FETCH / WRITE PMC passes (its solve with
# and without the fold: the prologue's extra bytes), and headline-kernel A/Bs (sum_stride, avg_every).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
export SWEEP_ONLY_FOLD=1 SWEEP_FOLD_CASES=1000000x100
timeout -k 10 300 python -u tools/ph_update_sweep.py $O/fold.json > $O/fold.log 2>&1 || { tail -5 $O/fold.log; exit 1; }
grep -v amdgpu $O/fold.log
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/ph_update_sweep.py > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/ph_update_sweep.py > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
python3 tools/fold_traffic.py $O/fetch $O/write $O/fold_traffic.json || exit 1
unset SWEEP_ONLY_FOLD SWEEP_FOLD_CASES
for v in "PHG_SUM_STRIDE=1" "PHG_SUM_STRIDE=2" "PHG_AVG_EVERY=4" "PHG_AVG_EVERY=8" "PHG_SUM_STRIDE=1"; do
  env $v timeout -k 10 200 python3 -u bench.py --conv-iters 20000 --cpu-seconds 0 > $O/ab.json 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab.json')); r=d['roofline']; t=d['time_to_conv']; print('$v', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'])"
done
