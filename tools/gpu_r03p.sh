# Round 3: UC with the local columns' primal step in the second hop: the block / border match test
# (same bits), the full-size UC tests, the UC bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -k "border or uc" -v --timeout 600 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --case uc --conv-time 60 --cpu-seconds 0 > $O/uc.json 2> $O/uc.err || { tail -5 $O/uc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/uc.json')); r=d['roofline']; t=d.get('time_to_conv') or {}; print('uc', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], r['max_pdhg_iters'], t.get('conv'), t.get('ph_iters'), t.get('seconds'))"
