# Round 3: netdes on row segments (delta form + unit codes + DPP row sums in 16-lane segments) --
# the netdes / block / bound tests, then A/B against PHG_BLOCK_SEG=0
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_fullsize.py tests/test_safe_bounds.py -k "netdes or border or sslp" -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|passed|failed|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit 1
for g in 1 0 1 0; do
  PHG_BLOCK_SEG=$g timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case netdes --scen 1024 > $O/nd_$g.json 2> $O/nd_$g.err || { tail -3 $O/nd_$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/nd_$g.json')); r=d['roofline']; print('netdes SEG=$g', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), d['config'].get('values'))"
done
