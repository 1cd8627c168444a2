# round 6: one-hop HEADX -- tests, then 10k / 1250 A/B with the kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_i; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() {  # tag env bench-args
  tag=$1; shift; envv=$1; shift
  env $envv timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d.get('time_to_conv',{}); r=d['roofline']
print('$tag', d['ms_per_step'], r.get('avg_launch_ms'), d.get('host_and_exchange_ms_per_step'), t.get('seconds'), t.get('ph_iters'))"
}
b s10k_oh1 PHG_HEADX_ONEHOP=1
b s10k_oh0 PHG_HEADX_ONEHOP=0
b s10k_oh1b PHG_HEADX_ONEHOP=1
b s10k_oh0b PHG_HEADX_ONEHOP=0
b s1250_oh1 PHG_HEADX_ONEHOP=1 --scen 1250 --conv-iters 0
b s1250_oh0 PHG_HEADX_ONEHOP=0 --scen 1250 --conv-iters 0
b s1250_oh1b PHG_HEADX_ONEHOP=1 --scen 1250 --conv-iters 0
b s1250_oh0b PHG_HEADX_ONEHOP=0 --scen 1250 --conv-iters 0
for v in 0 1; do
PHG_HEADX_ONEHOP=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof10k_$v -o run -- python3 bench.py --steps 40 --warmup 5 --conv-iters 0 --cpu-seconds 0 > $O/prof10k_$v.log 2>&1 || { tail -5 $O/prof10k_$v.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -c1-150 $f | grep -E "node_sums|schedule"; done
