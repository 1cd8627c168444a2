# round 6: full GPU suite after the node-sum head changes, then 10k / 1250 bench + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_k; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large.py tests/test_gpu_loop.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head -20; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() {  # tag env bench-args
  tag=$1; shift; envv=$1; shift
  env $envv timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d.get('time_to_conv',{}); r=d['roofline']
print('$tag', d['ms_per_step'], r.get('avg_launch_ms'), d.get('host_and_exchange_ms_per_step'), t.get('seconds'), t.get('ph_iters'))"
}
b s10k_a X=0
b s10k_b X=0
b s1250_a X=0 --scen 1250 --conv-iters 0
b s1250_b X=0 --scen 1250 --conv-iters 0
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof10k -o run -- python3 bench.py --steps 40 --warmup 5 --conv-iters 0 --cpu-seconds 0 > $O/prof10k.log 2>&1 || { tail -5 $O/prof10k.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1250 -o run -- python3 bench.py --scen 1250 --steps 40 --warmup 5 --conv-iters 0 --cpu-seconds 0 > $O/prof1250.log 2>&1 || { tail -5 $O/prof1250.log; exit 1; }
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -c1-150 $f | grep -E "node_sums|schedule"; done
