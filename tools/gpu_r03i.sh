# Round 3: fold diagnosis vs host W, the delta form with on-the-fly scaling (netdes), the wave kernel
# at 2 waves per SIMD (sslp) vs the block kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 120 python -u tools/fold_diag.py 4 1 2 > $O/fold_diag.log 2>&1; echo "fold_diag exit $?"; grep -v amdgpu.ids $O/fold_diag.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -k "wave or delta or netdes or border" -v -s --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|wave / block|^E  " $O/tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
line() {  # name json
  python3 -c "import json; d=json.load(open('$2')); r=d['roofline']; t=d.get('time_to_conv') or {}; print('$1', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['frac'], r.get('hbm_measured_GBs'), d['config']['pdhg_layout'], d['config'].get('values'), t.get('conv'), t.get('ph_iters'), t.get('seconds'))"
}
timeout -k 10 400 python3 -u bench.py --conv-time 60 --cpu-seconds 0 --case netdes --scen 1024 > $O/netdes.json 2> $O/netdes.err || exit 1
line delta $O/netdes.json
timeout -k 10 300 python3 -u bench.py --conv-iters 0 --cpu-seconds 0 --case sslp --scen 4096 > $O/sslp.json 2> $O/sslp.err || exit 1
line wave2 $O/sslp.json
timeout -k 10 300 python3 -u bench.py --conv-iters 0 --cpu-seconds 0 --case sslp --scen 4096 --layout block > $O/sslp_block.json 2> $O/sslp_block.err || exit 1
line block $O/sslp_block.json
