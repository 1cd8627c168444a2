# A/B of the persistent lane-local kernel (PHG_LOCAL_PERSIST=1, default) vs one item per group (0):
# local-layout parity tests, then bench lines (no conv / cpu legs) for both
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "local or pipelined" > gpurun_out/persist_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/persist_tests.log
[ $rc -eq 0 ] || exit $rc
for P in 1 0 1 0; do
  PHG_LOCAL_PERSIST=$P timeout -k 10 200 python -u bench.py --conv-iters ${CONV_ITERS:-0} --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/bench_p$P.json 2> gpurun_out/bench_p$P.err
  rc=$?; echo "persist=$P exit $rc"; python -c "import json; d=json.load(open('gpurun_out/bench_p$P.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'], d.get('time_to_conv',{}).get('seconds'))"
  [ $rc -eq 0 ] || exit $rc
done
