set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_gpu_f4.py tests/test_gpu_loop.py tests/test_gpu_cylinders.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03c/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03c/tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 2; do
  PHG_SUM_STRIDE=$v timeout -k 10 200 python -u bench.py --cpu-seconds 0 --conv-iters 20000 > gpurun_out/r03c/bench_s$v.json 2> gpurun_out/r03c/bench_s$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r03c/bench_s$v.json')); r=d['roofline']; t=d['time_to_conv']; print('stride $v', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'], t['rel_gap_Eobj_vs_ef'])"
done
timeout -k 10 300 python -u tools/lagr_diag.py 1000 200000 gpurun_out/diag/lagr1000w.npz || exit $?
timeout -k 10 300 python -u tools/lagr_diag.py 10000 20000 gpurun_out/diag/lagr10000w.npz || exit $?
