# Node-segment cap A/B for the PH update at S*N = 1e7 / 1e8 (PHG_NODESEG_MAX), one process each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for V in 128 512 2048 8192; do
  PHG_NODESEG_MAX=$V timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0, 'tools'); sys.argv = ['x']
import ph_update_sweep as m
for S, N in ((100000, 100), (100000, 1000)):
    r = m.run(S, N)
    print('seg_max $V', S, N, r['avg_us'], r['frac_hbm'], r['check_ok'], flush=True)
" 2>&1 | grep -v amdgpu.ids
  rc=$?; [ $rc -eq 0 ] || exit $rc
done
