# Round 3: lane-local kernel cycle split with the check's KKT part (products + reductions) separated
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ai
mkdir -p $O
PHG_LOCAL_PROF=1 timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 > $O/prof.json 2> $O/prof.err || { tail -3 $O/prof.err; exit 1; }
grep PHG_LOCAL_PROF $O/prof.err | tail -3
