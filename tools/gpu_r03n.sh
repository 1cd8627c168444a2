# Round 3: UC (overlapped exchange) Lagrangian test with safe_bound 1 / 2, the UC bench line and its
# trace (PHG_COOP=0), then sslp 4096 with the row piece sums issued together (PHG_PSUM=1) vs default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -k "lagrangian or sslp" -v -s --timeout 500 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " $O/tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --case uc --conv-time 60 --cpu-seconds 0 > $O/uc.json 2> $O/uc.err || { tail -5 $O/uc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/uc.json')); r=d['roofline']; t=d.get('time_to_conv') or {}; print('uc', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'], t.get('conv'), t.get('ph_iters'), t.get('seconds'))"
PHG_COOP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/uc_trace -o run -- python3 bench.py --case uc --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds 0 > $O/uc_trace.log 2>&1
echo "uc rocprof (PHG_COOP=0) exit $?"
for v in 0 1 0 1; do
  PHG_PSUM=$v timeout -k 10 300 python3 -u bench.py --conv-iters 0 --cpu-seconds 0 --case sslp --scen 4096 > $O/sslp.json 2> $O/sslp.err || { tail -3 $O/sslp.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sslp.json')); r=d['roofline']; print('PSUM=$v', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['frac'])"
done
