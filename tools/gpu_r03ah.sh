# Round 3: lane-local prologue with its loads batched -- cycle split and the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
PHG_LOCAL_PROF=1 timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 > $O/prof.json 2> $O/prof.err || { tail -3 $O/prof.err; exit 1; }
grep PHG_LOCAL_PROF $O/prof.err | tail -3
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --conv-iters 20000 --cpu-seconds 0 > $O/b_$i.json 2> $O/b_$i.err || { tail -3 $O/b_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$i.json')); r=d['roofline']; t=d['time_to_conv']; print('farmer', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'], t['rel_gap_Eobj_vs_ef'])"
done
