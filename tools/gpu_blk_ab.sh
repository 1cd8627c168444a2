set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 200 --timeout-method thread -m gpu -k "block" > gpurun_out/blk_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -8 gpurun_out/blk_tests.log
[ $rc -eq 0 ] || exit $rc
for E in PHG_BLOCK_STREAM=1 PHG_BLOCK_STREAM=0; do
  env $E timeout -k 10 200 python -u bench.py --case sslp --scen 4096 --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 > gpurun_out/blk_$E.json 2> gpurun_out/blk_$E.err
  rc=$?; [ $rc -eq 0 ] || { echo "[$E] exit $rc"; tail -5 gpurun_out/blk_$E.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/blk_$E.json')); r=d['roofline']; print('[$E]', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'])"
done
