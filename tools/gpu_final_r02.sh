# End-of-session refresh (round 2): every -m gpu test, smoke, the default bench line with its
# kernel-trace + PMC profiles, then the secondary cases (sslp, netdes, hydro) with their PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_round_profile.sh > gpurun_out/round_profile.log 2>&1
rc=$?; echo "round profile exit $rc"; tail -2 gpurun_out/round_profile.log | head -c 600; echo; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_cases_r02.sh
