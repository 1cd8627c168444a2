set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag gpurun_out/r03b
timeout -k 10 300 python -u tools/lagr_diag.py 1000 200000 gpurun_out/diag/lagr1000w.npz || exit $?
timeout -k 10 300 python -u tools/lagr_diag.py 10000 20000 gpurun_out/diag/lagr10000w.npz || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_f4.py tests/test_gpu_loop.py tests/test_gpu_cylinders.py -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03b/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r03b/tests.log | tail -40
