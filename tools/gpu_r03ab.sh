# Round 3: sslp block kernel with row segments (DPP row sums, two barriers per PDHG iteration) --
# the sslp / block tests, then A/B against PHG_BLOCK_SEG=0 at 4 096 scenarios
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "sslp or wave" -v --timeout 250 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest sslp exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit 1
for g in 1 0 1 0; do
  PHG_BLOCK_SEG=$g timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case sslp --scen 4096 > $O/sslp_$g.json 2> $O/sslp_$g.err || { tail -3 $O/sslp_$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sslp_$g.json')); r=d['roofline']; print('sslp SEG=$g', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), d['config'].get('kernel_variant'), r.get('kernel'))"
done
