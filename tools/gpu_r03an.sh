# Round 3: row segments with non-owner lanes' sums zeroed -- block tests, sslp and netdes benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03an
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_fullsize.py tests/test_safe_bounds.py -k "netdes or sslp or wave or register" -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -6
[ $rc -eq 0 ] || exit 1
for c in "sslp --scen 4096" "netdes --scen 1024"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case $c > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'))"
done
