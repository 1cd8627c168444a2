# round 6 end: the whole GPU suite, then the round profile (kernel trace, FETCH / WRITE passes, full bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_final
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r06_final/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/r06_final/tests.log | head; tail -1 gpurun_out/r06_final/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_round_profile.sh
