# round 6: launch schedule A/B after batching its loads -- bench 10k / 1250 both ways + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_g; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_loop.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() {  # tag env bench-args
  tag=$1; shift; envv=$1; shift
  env $envv timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d.get('time_to_conv',{}); r=d['roofline']
print('$tag', d['ms_per_step'], r.get('avg_launch_ms'), d.get('host_and_exchange_ms_per_step'), t.get('seconds'), t.get('ph_iters'))"
}
b fuse1_a PHG_SCHED_FUSE=1
b fuse0_a PHG_SCHED_FUSE=0
b fuse1_b PHG_SCHED_FUSE=1
b fuse0_b PHG_SCHED_FUSE=0
b s1250_fuse1 PHG_SCHED_FUSE=1 --scen 1250 --conv-iters 0
b s1250_fuse0 PHG_SCHED_FUSE=0 --scen 1250 --conv-iters 0
for f in 0 1; do
  PHG_SCHED_FUSE=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$f -o run -- python3 bench.py --steps 40 --warmup 5 --conv-iters 0 --cpu-seconds 0 > $O/prof$f.log 2>&1 || { tail -5 $O/prof$f.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -c1-150 $f | head -8; done
