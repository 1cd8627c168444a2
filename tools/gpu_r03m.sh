# Round 3: sslp 4096 row piece sums issued together (PHG_PSUM=1) vs the default, alternating runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "sslp and prox" -v --timeout 200 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  PHG_PSUM=$v timeout -k 10 300 python3 -u bench.py --conv-iters 0 --cpu-seconds 0 --case sslp --scen 4096 > $O/sslp.json 2> $O/sslp.err || { tail -3 $O/sslp.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sslp.json')); r=d['roofline']; print('PSUM=$v', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['frac'])"
done
