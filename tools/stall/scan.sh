# stall scan over a long farmer 10k PH trajectory, then the default bench line with its conv leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/stall2; mkdir -p $O
STALL_K=400 timeout -k 10 400 python -u tools/stall/find_stall.py > $O/scan.log 2>&1 || { tail -5 $O/scan.log; exit 1; }
echo "steps with a stall: $(grep -c STALL $O/scan.log)"; grep STALL $O/scan.log | head -5; tail -2 $O/scan.log
timeout -k 10 400 python -u bench.py --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read()); r=d['roofline']; t=d['time_to_conv']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['pdhg_iters_per_scen_per_step'], t['seconds'], t['ph_iters'], t['conv'], t.get('rel_gap_Eobj_vs_ef'), t.get('rel_gap_inner_vs_ef'))"
