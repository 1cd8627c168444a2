# Round 3: fold diagnosis (xN vs xs dc), wave-vs-block and netdes delta tests, netdes delta (PMC +
# bench) against PHG_DELTA=0 with constant-entry scaling, sslp 4096 wave (PMC + bench) vs block.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 120 python -u tools/fold_diag.py 4 1 3 > $O/fold_diag.log 2>&1; echo "fold_diag exit $?"; grep -v amdgpu.ids $O/fold_diag.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -k "wave or delta" -v -s --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|wave / block|^E  " $O/tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
pmc() {   # name layout args...
  local nm=$1 lay=$2; shift 2
  local B="bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 $*"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$nm/fetch -o run -- python3 $B > $O/$nm.fetch.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$nm/write -o run -- python3 $B > $O/$nm.write.log 2>&1 || return 1
  python3 tools/traffic_from_pmc.py $O/$nm/fetch/run_counter_collection.csv $O/$nm/write/run_counter_collection.csv $lay $O/${nm}_traffic.json $nm "$*" > /dev/null || return 1
}
line() {  # name json
  python3 -c "import json; d=json.load(open('$2')); r=d['roofline']; t=d.get('time_to_conv') or {}; print('$1', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['frac'], r.get('hbm_measured_GBs'), d['config']['pdhg_layout'], d['config'].get('values'), t.get('conv'), t.get('ph_iters'), t.get('seconds'))"
}
pmc netdes block --case netdes --scen 1024 || exit 1
timeout -k 10 400 python3 -u bench.py --traffic-json $O/netdes_traffic.json --conv-time 60 --cpu-seconds 0 --case netdes --scen 1024 > $O/netdes.json 2> $O/netdes.err || exit 1
line delta $O/netdes.json
pmc sslp wave --case sslp --scen 4096 || exit 1
timeout -k 10 400 python3 -u bench.py --traffic-json $O/sslp_traffic.json --conv-time 60 --cpu-seconds 0 --case sslp --scen 4096 > $O/sslp.json 2> $O/sslp.err || exit 1
line wave $O/sslp.json
timeout -k 10 400 python3 -u bench.py --conv-time 60 --cpu-seconds 0 --case sslp --scen 4096 --layout block > $O/sslp_block.json 2> $O/sslp_block.err || exit 1
line block $O/sslp_block.json
