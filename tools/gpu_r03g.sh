# Round 3: fold bit-identity diagnosis, the large-subproblem tests (delta value form), and netdes 1024
# with the delta form (PMC FETCH/WRITE passes + bench line) against PHG_DELTA=0.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 120 python -u tools/fold_diag.py 4 1 40 > $O/fold_diag.log 2>&1; echo "fold_diag exit $?"; cat $O/fold_diag.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -k "netdes or border or pipelined or folded" -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case netdes --scen 1024"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/netdes/fetch -o run -- python3 $B > $O/netdes.fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/netdes/write -o run -- python3 $B > $O/netdes.write.log 2>&1 || exit 1
python3 tools/traffic_from_pmc.py $O/netdes/fetch/run_counter_collection.csv $O/netdes/write/run_counter_collection.csv block $O/netdes_traffic.json netdes "--case netdes --scen 1024" > /dev/null || exit 1
cat $O/netdes_traffic.json
timeout -k 10 400 python3 -u bench.py --traffic-json $O/netdes_traffic.json --conv-time 60 --cpu-seconds 0 --case netdes --scen 1024 > $O/netdes.json 2> $O/netdes.err || exit 1
python3 -c "import json; d=json.load(open('$O/netdes.json')); r=d['roofline']; print('delta', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r.get('hbm_measured_GBs'), d['config']['values'], d.get('time_to_conv', {}).get('conv'), d.get('time_to_conv', {}).get('ph_iters'))"
PHG_DELTA=0 timeout -k 10 400 python3 -u bench.py --conv-time 60 --cpu-seconds 0 --case netdes --scen 1024 > $O/netdes_off.json 2> $O/netdes_off.err || exit 1
python3 -c "import json; d=json.load(open('$O/netdes_off.json')); r=d['roofline']; print('off', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], d['config']['values'], d.get('time_to_conv', {}).get('conv'), d.get('time_to_conv', {}).get('ph_iters'))"
# the one-wave-per-scenario shared-matrix kernel (sslp): parity tests, then sslp 4096 wave vs block
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_fullsize.py -k "sslp or wave" -v --timeout 300 --timeout-method thread -m gpu > $O/tests_wave.log 2>&1
rc=$?; echo "pytest wave exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|wave / block" $O/tests_wave.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for L in wave block; do
  timeout -k 10 300 python3 -u bench.py --conv-iters 0 --cpu-seconds 0 --case sslp --scen 4096 --layout $L > $O/sslp_$L.json 2> $O/sslp_$L.err || { tail -5 $O/sslp_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sslp_$L.json')); r=d['roofline']; print('$L', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['frac'], d['config']['pdhg_layout'])"
done
