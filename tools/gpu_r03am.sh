# Round 3: unit codes as LDS byte addresses (sign from bit 0): netdes tests (unit = delta form bit
# for bit), then the netdes bench x2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03am
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_fullsize.py tests/test_safe_bounds.py -k "netdes" -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -6
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case netdes --scen 1024 > $O/nd_$i.json 2> $O/nd_$i.err || { tail -3 $O/nd_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/nd_$i.json')); r=d['roofline']; print('netdes', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), d['config'].get('values'))"
done
