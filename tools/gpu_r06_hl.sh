# round 6: hydro on the lane-local layout (16 lanes / scenario, every row a coupling row)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_hl; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hydro" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
for sc in 500 2000 4000; do
  for lay in gather local; do
    timeout -k 10 200 python -u bench.py --case hydro --scen $sc --layout $lay --cpu-seconds 0 > $O/hydro_${sc}_$lay.json 2> $O/hydro_${sc}_$lay.err || { tail -3 $O/hydro_${sc}_$lay.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/hydro_${sc}_$lay.json').read().strip().splitlines()[-1]); t=d['time_to_conv']; print('hydro $sc $lay', d['config']['pdhg_layout'], d['value'], d['ms_per_step'], t['seconds'], t['ph_iters'], t['conv'], d.get('pdhg_iters_per_solve'))"
  done
done
