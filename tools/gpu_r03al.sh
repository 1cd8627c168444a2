set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "register_pieces or sslp or wave or netdes" -v --timeout 250 --timeout-method thread -m gpu > gpurun_out/r03al.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03al.log | tail -10
