# Round 3: the full -m gpu suite, netdes row piece sums issued together (PHG_PSUM) A/B, then the
# round profile (kernel trace + FETCH/WRITE PMC + the default bench line with that traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -v --timeout 600 --timeout-method thread -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 0 1 0; do
  PHG_PSUM=$v timeout -k 10 300 python3 -u bench.py --conv-iters 0 --cpu-seconds 0 --case netdes --scen 1024 > $O/netdes.json 2> $O/netdes.err || { tail -3 $O/netdes.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/netdes.json')); r=d['roofline']; print('PSUM=$v', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'])"
done
bash tools/gpu_round_profile.sh || exit $?
