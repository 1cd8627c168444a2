# Round 3: lane-local epilogue without global loads (dc in LDS, indices in registers): cycle split,
# farmer / fold / north-star tests, headline bench x2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
PHG_LOCAL_PROF=1 timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 > $O/prof.json 2> $O/prof.err || { tail -3 $O/prof.err; exit 1; }
grep PHG_LOCAL_PROF $O/prof.err | tail -3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py tests/test_gpu_fullsize.py tests/test_gpu_loop.py -k "farmer or fold or northstar or converged or loop" -v --timeout 400 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -6
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --conv-iters 20000 --cpu-seconds 0 > $O/b_$i.json 2> $O/b_$i.err || { tail -3 $O/b_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$i.json')); r=d['roofline']; t=d['time_to_conv']; print('farmer', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'], t['rel_gap_Eobj_vs_ef'])"
done
