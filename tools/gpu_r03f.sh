# Round 3 re-entry: the full -m gpu suite, the round profile (kernel trace + FETCH/WRITE PMC passes +
# the default bench line with that traffic), then the PH-update sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03f
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03f/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03f/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_round_profile.sh || exit $?
timeout -k 10 400 python -u tools/ph_update_sweep.py gpurun_out/r03f/sweep.json > gpurun_out/r03f/sweep.log 2>&1 || exit $?
cat gpurun_out/r03f/sweep.log
