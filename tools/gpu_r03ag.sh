# Round 3: cycle split of the lane-local kernel (PHG_LOCAL_PROF=1) on the headline workload, check
# intervals 32 and 64
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
for c in 32 64; do
  PHG_LOCAL_PROF=1 timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --check-every $c > $O/f_$c.json 2> $O/f_$c.err || { tail -3 $O/f_$c.err; exit 1; }
  echo "check_every=$c"; grep PHG_LOCAL_PROF $O/f_$c.err | tail -4
done
