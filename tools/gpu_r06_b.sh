# round 6: new GPU tests, hydro layout by scenario count, UC eps-schedule variants
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_schedule.py tests/test_gpu_large.py -k "heldout or schedule" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
for sc in 500 2000 4000; do
  for lay in auto mfma; do
    timeout -k 10 200 python -u bench.py --case hydro --scen $sc --layout $lay --cpu-seconds 0 > $O/hydro_${sc}_$lay.json 2> $O/hydro_${sc}_$lay.err || { tail -3 $O/hydro_${sc}_$lay.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/hydro_${sc}_$lay.json').read().strip().splitlines()[-1]); t=d['time_to_conv']; print('hydro $sc $lay', d['config']['pdhg_layout'], d['value'], d['ms_per_step'], t['seconds'], t['ph_iters'], t['conv'])"
  done
done
for X in "1e-2:1e-5,3e-4:1e-6,0:1e-7" "1e-2:1e-5,1e-3:1e-6,2e-4:3e-7,0:1e-7"; do
  tag=$(echo $X | tr ':,' '__')
  timeout -k 10 420 python -u bench.py --case uc --uc-rho cost --steps 3 --warmup 1 --cpu-seconds 0 --conv-time 120 --eps-schedule $X > $O/uc_$tag.json 2> $O/uc_$tag.err || { tail -5 $O/uc_$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/uc_$tag.json').read().strip().splitlines()[-1]); t=d['time_to_conv']
print('uc $X', t['seconds'], t['ph_iters'], t['conv'], t.get('seconds_iter0_and_first_20_ph_iters'), t.get('final_pdhg_eps'), t.get('Eobj'))"
done
