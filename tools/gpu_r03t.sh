# Round 3: the UC case's per-scenario PDHG iteration tail (what sets the bordered kernel's launch time)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
PHG_COOP=0 timeout -k 10 500 python3 -u tools/uc_iter_tail.py 64 8 1e-6 > $O/uc_tail.log 2>&1
rc=$?; echo "uc_iter_tail exit $rc"; cat $O/uc_tail.log | tail -12
