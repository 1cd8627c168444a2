# Full round check on the GPU box: every -m gpu test, smoke, one default bench line.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -8 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
