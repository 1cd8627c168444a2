# Round 3: the unit form of the netdes delta kernel (constant entries +-1, matrix held in LDS as
# 16-bit entry codes) -- parity (same bits as the delta form) and the netdes bench, A/B against
# PHG_UNIT=0; then the other workgroup-layout tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "netdes_delta" -v --timeout 250 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest netdes_delta exit $rc"; grep -E "FAILED|passed|failed|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit 1
for u in 1 0 1 0; do
  PHG_UNIT=$u timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case netdes --scen 1024 > $O/nd_$u.json 2> $O/nd_$u.err || { tail -3 $O/nd_$u.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/nd_$u.json')); r=d['roofline']; print('PHG_UNIT=$u', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), r.get('pdhg_iters_per_scen_per_step'), d['config'].get('values'))"
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_fullsize.py tests/test_safe_bounds.py -k "netdes or sslp or border" -v --timeout 250 --timeout-method thread -m gpu > $O/tests2.log 2>&1
rc=$?; echo "pytest block/netdes exit $rc"; grep -E "FAILED|passed|failed" $O/tests2.log | tail -8
