# Block-kernel A/B: block-layout GPU tests, then sslp / netdes bench lines per env setting in $ENVS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 200 --timeout-method thread -m gpu -k "block" > gpurun_out/blk_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/blk_tests.log
[ $rc -eq 0 ] || exit $rc
i=0
for C in ${CASES:-"sslp:4096"}; do
for E in ${ENVS:-PHG_AVG_EVERY=6}; do
  i=$((i+1)); cs=${C%%:*}; sc=${C##*:}
  env $E timeout -k 10 200 python -u bench.py --case $cs --scen $sc --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 > gpurun_out/blk_$i.json 2> gpurun_out/blk_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "[$C $E] exit $rc"; tail -5 gpurun_out/blk_$i.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/blk_$i.json')); r=d['roofline']; print('[$C $E]', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'])"
done
done
