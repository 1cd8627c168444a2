# Secondary workloads of SURVEY 8(d) (M1 rho=0.1, M2 sslp sizes, M3 hydro trees, M4 netdes sizes):
# one bench line each into gpurun_out/cases/.  Each step has its own time limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cases
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/cases/dist_tests.log 2>&1
rc=$?; echo "dist tests exit $rc"; tail -30 gpurun_out/cases/dist_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 ${T:-300} python -u bench.py --conv-time 60 --cpu-seconds 6 "$@" > gpurun_out/cases/$nm.json 2> gpurun_out/cases/$nm.err
  local rc=$?; echo "$nm exit $rc"; tail -2 gpurun_out/cases/$nm.err; head -c 600 gpurun_out/cases/$nm.json; echo
  return $rc
}
run sslp8192 --case sslp --scen 8192 --conv-iters 0 && \
T=400 run sslp4096 --case sslp --scen 4096 --conv-time 100 && \
run netdes4096 --case netdes --scen 4096 --conv-iters 0 --cpu-seconds 0
