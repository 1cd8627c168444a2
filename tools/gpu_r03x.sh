# Round 3: the size-based primal-weight theta default (UC 0.05, netdes 0.5) -- UC tail over 20 PH
# iterations (default and 0.02), UC and netdes benches with time to conv, then the UC / netdes /
# border / bound tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
PHG_COOP=0 timeout -k 10 300 python3 -u tools/uc_iter_tail.py 64 20 1e-6 > $O/uc_tail_default.log 2>&1 || { tail -3 $O/uc_tail_default.log; exit 1; }
grep -E "SUMMARY|PH 20" $O/uc_tail_default.log
UC_OPTS='{"pdhg_primal_weight_theta": 0.02}' PHG_COOP=0 timeout -k 10 300 python3 -u tools/uc_iter_tail.py 64 20 1e-6 > $O/uc_tail_002.log 2>&1 || { tail -3 $O/uc_tail_002.log; exit 1; }
grep SUMMARY $O/uc_tail_002.log
for c in uc netdes; do
  timeout -k 10 300 python3 -u bench.py --case $c --conv-time 60 --cpu-seconds 0 > $O/$c.json 2> $O/$c.err || { tail -3 $O/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; t=d['time_to_conv']; print('$c', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), r.get('max_pdhg_iters'), t['seconds'], t['ph_iters'], t.get('conv'), t.get('converged'))"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py tests/test_safe_bounds.py tests/test_gpu_fullsize.py -v --timeout 400 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -10
