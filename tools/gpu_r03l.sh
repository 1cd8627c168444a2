# Round 3: the UC bordered kernel with the linking-row exchange overlapped (same bits: the block /
# border match test), the full-size UC tests, and the UC bench line (S = 64) with its trace (PHG_COOP=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -k "border or uc" -v -s --timeout 600 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --case uc --conv-time 60 --cpu-seconds 0 > $O/uc.json 2> $O/uc.err || { tail -5 $O/uc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/uc.json')); r=d['roofline']; t=d.get('time_to_conv') or {}; print('uc', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'], t.get('conv'), t.get('ph_iters'), t.get('seconds'))"
PHG_COOP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/uc_trace -o run -- python3 bench.py --case uc --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds 0 > $O/uc_trace.log 2>&1
echo "uc rocprof (PHG_COOP=0) exit $?"
