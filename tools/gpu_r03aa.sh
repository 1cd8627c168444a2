# Round 3: sslp block kernel with a register budget for 3 / 4 waves per SIMD (PHG_BLOCK_MINW)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
for w in 1 3 4 1 3 4; do
  PHG_BLOCK_MINW=$w timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case sslp --scen 4096 > $O/sslp_$w.json 2> $O/sslp_$w.err || { tail -3 $O/sslp_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sslp_$w.json')); r=d['roofline']; print('sslp MINW=$w', d['value'], d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), d['config'].get('kernel_variant', ''))"
done
PHG_BLOCK_MINW=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_fullsize.py -k "sslp" -v --timeout 250 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest sslp MINW=3 exit $rc"; grep -E "FAILED|passed|failed" $O/tests.log | tail -5
