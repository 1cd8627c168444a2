# round 6: netdes block kernel with q in LDS / SGPR piece offsets (libphg_blkab.so) vs HEAD (libphg.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_m; mkdir -p $O
NEW=$GRAFT_REPO_ROOT/mpi-sppy_amd/libphg_blkab.so
PHG_LIB=$NEW timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ -k "netdes or block_kernel or sslp" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" $O/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
b() {  # tag env bench-args
  tag=$1; shift; envv=$1; shift
  env $envv timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d.get('time_to_conv',{}); r=d['roofline']
print('$tag', d['ms_per_step'], r.get('avg_launch_ms'), r.get('pdhg_iters_per_scen_per_step'), t.get('seconds'), t.get('ph_iters'))"
}
for rep in 1 2; do
  b net_new_$rep PHG_LIB=$NEW --case netdes --conv-iters 0
  b net_old_$rep X=0 --case netdes --conv-iters 0
done
b sslp_new PHG_LIB=$NEW --case sslp --conv-iters 0
b sslp_old X=0 --case sslp --conv-iters 0
