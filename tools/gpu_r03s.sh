# Round 3: the packed lane-local layout (two farmer crops per lane, 16 lanes per scenario, four
# scenarios per wave; PHG_LOCAL_PACK=1) -- parity tests under it, then headline A/B against the
# default 32-lane layout with time to conv.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
PHG_LOCAL_PACK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "farmer" -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest (packed) exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  PHG_LOCAL_PACK=$v timeout -k 10 200 python3 -u bench.py --conv-iters 20000 --cpu-seconds 0 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -3 $O/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab_$v.json')); r=d['roofline']; t=d['time_to_conv']; print('PACK=$v', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'], t['rel_gap_Eobj_vs_ef'], d['config'].get('kernel', ''))"
done
