# A/B of environment switches: ENVS=';'-separated env assignments (e.g. "PHG_LOCAL_GENERIC=1;PHG_LOCAL_GENERIC=0"),
# each run twice, interleaved; local-layout parity tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu ${TESTK:+-k "$TESTK"} > gpurun_out/envab_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/envab_tests.log
[ $rc -eq 0 ] || exit $rc
IFS=';' read -ra SETS <<< "$ENVS"
for rep in 1 2; do
i=0
for E in "${SETS[@]}"; do
  i=$((i+1))
  env $E timeout -k 10 200 python -u bench.py --conv-iters ${CONV_ITERS:-0} --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/envab_$i.json 2> gpurun_out/envab_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "[$E] exit $rc"; tail -5 gpurun_out/envab_$i.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/envab_$i.json')); r=d['roofline']; print('[$E]', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'], d.get('time_to_conv',{}).get('seconds'))"
done
done
