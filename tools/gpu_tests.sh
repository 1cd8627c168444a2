set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu1.log 2>&1
echo "pytest exit $?"
tail -40 gpurun_out/gpu1.log
