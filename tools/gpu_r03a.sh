# Round 3, first GPU pass: safe bounds, gap-with-constant termination, split PH-update timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests/test_gpu_cylinders.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_northstar.py -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03a/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r03a/tests.log | tail -80
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-seconds 10 > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
rc=$?; echo "bench exit $rc"; tail -3 gpurun_out/r03a/bench.err; cat gpurun_out/r03a/bench.json
