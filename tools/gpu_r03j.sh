# Round 3: the folded update after the FMA-contraction fix (diag + the fold tests); netdes delta PMC +
# bench; the north-star and full-size tests with their printed numbers; the rocprofv3 teardown
# segfault: the cooperative-launch repro and UC profiled with PHG_COOP=0.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 120 python -u tools/fold_diag.py 4 1 30 > $O/fold_diag.log 2>&1; echo "fold_diag exit $?"; grep -v amdgpu.ids $O/fold_diag.log | tail -4
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py tests/test_gpu_fullsize.py -k "pipelined or folded or northstar or converged or full_size" -v -s --timeout 400 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Lagrangian|first stage|^E  " $O/tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case netdes --scen 1024"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/netdes/fetch -o run -- python3 $B > $O/netdes.fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/netdes/write -o run -- python3 $B > $O/netdes.write.log 2>&1 || exit 1
python3 tools/traffic_from_pmc.py $O/netdes/fetch/run_counter_collection.csv $O/netdes/write/run_counter_collection.csv block $O/netdes_traffic.json netdes "--case netdes --scen 1024" > /dev/null || exit 1
timeout -k 10 400 python3 -u bench.py --traffic-json $O/netdes_traffic.json --conv-time 60 --cpu-seconds 6 --case netdes --scen 1024 > $O/netdes.json 2> $O/netdes.err || exit 1
python3 -c "import json; d=json.load(open('$O/netdes.json')); r=d['roofline']; print('netdes', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['frac'], r.get('hbm_measured_GBs'), r.get('traffic'))"
make -C tools/repro coop_exit > /dev/null 2>&1 || hipcc --offload-arch=gfx950 -O2 tools/repro/coop_exit.hip -o tools/repro/coop_exit || exit 1
for mode in 0 1; do
  timeout -k 10 60 ./tools/repro/coop_exit $mode; echo "plain mode $mode exit $?"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/coop$mode -o run -- ./tools/repro/coop_exit $mode > $O/coop$mode.log 2>&1
  echo "rocprofv3 mode $mode exit $?"; grep -E "mode|SIGSEGV|Segmentation|Aborted" $O/coop$mode.log | head -3
done
PHG_COOP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/uc_trace -o run -- python3 bench.py --case uc --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds 0 > $O/uc_trace.log 2>&1
echo "uc rocprof (PHG_COOP=0) exit $?"; grep -E '"metric"' $O/uc_trace.log | python3 -c "import sys,json; [print('uc', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']) for d in map(json.loads, sys.stdin)]"
