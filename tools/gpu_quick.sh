# quick GPU check: parity tests, then bench lines for both PDHG layouts (no conv / cpu legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -30 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for L in ${LAYOUTS:-gather local}; do
  timeout -k 10 200 python -u bench.py --layout $L --conv-iters ${CONV_ITERS:-0} --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/bench_$L.json 2> gpurun_out/bench_$L.err
  rc=$?; echo "bench $L exit $rc"; tail -3 gpurun_out/bench_$L.err; cat gpurun_out/bench_$L.json
  [ $rc -eq 0 ] || exit $rc
done
