set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03e/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03e/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mode in 0 1; do
  timeout -k 10 60 ./tools/repro/coop_exit $mode; echo "plain mode $mode exit $?"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03e/coop$mode -o run -- ./tools/repro/coop_exit $mode > gpurun_out/r03e/coop$mode.log 2>&1
  echo "rocprofv3 mode $mode exit $?"; grep -E "mode|SIGSEGV|Aborted" gpurun_out/r03e/coop$mode.log | head -3
done
