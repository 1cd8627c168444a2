# Round 3: the whole -m gpu suite and smoke(), as the driver runs them at round end
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; grep -E "FAILED|ERROR|passed|failed" $O/suite.log | tail -12
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke exit $?"; tail -3 $O/smoke.log
