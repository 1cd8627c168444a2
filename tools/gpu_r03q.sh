# Round 3: headline A/B of the windowed running sums (PHG_SUM_STRIDE=3) against the default, alternating,
# with time to conv; then the parity tests of the local kernel under the windowed sums.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
for v in 1 3 1 3; do
  PHG_SUM_STRIDE=$v timeout -k 10 200 python3 -u bench.py --conv-iters 20000 --cpu-seconds 0 > $O/ab.json 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab.json')); r=d['roofline']; t=d['time_to_conv']; print('SUM_STRIDE=$v', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'], t['rel_gap_Eobj_vs_ef'])"
done
PHG_SUM_STRIDE=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py tests/test_gpu_fullsize.py -k "farmer or prox or northstar or converged" -v --timeout 400 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest (windowed sums) exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -8
