# round 6: one-sided total-acreage coupling row in offset form for unfixed solves (libphg.so) vs the two-sided form (libphg_cone0.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_r; mkdir -p $O
OLD=$GRAFT_REPO_ROOT/mpi-sppy_amd/libphg_cone0.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_northstar.py tests/test_gpu_loop.py tests/test_gpu_fullsize.py tests/test_gpu_f4.py tests/test_gpu_cylinders.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
b() {  # tag env bench-args
  tag=$1; shift; envv=$1; shift
  env $envv timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d.get('time_to_conv',{}); r=d['roofline']
print('$tag', d['ms_per_step'], r.get('avg_launch_ms'), r.get('pdhg_iters_per_scen_per_step'), r.get('max_pdhg_iters'), t.get('seconds'), t.get('ph_iters'), t.get('gap_rel_to_ef') or t.get('ef_gap'))"
}
for rep in 1 2 3; do
  b new_$rep X=0
  b old_$rep PHG_LIB=$OLD
done
b new_1250 X=0 --scen 1250 --conv-iters 0
b old_1250 PHG_LIB=$OLD --scen 1250 --conv-iters 0
