# round 6: launch schedule in the node-sum launch (PHG_SCHED_FUSE) -- tests, then the 10k / 1250 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_f; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
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
