# round 6: secondary kernels' PMC -- hydro 2 000 (wave-gather) issue counters, netdes 1 024 (block) traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_sec; mkdir -p $O
H="python3 bench.py --case hydro --steps 10 --warmup 3 --conv-iters 0 --cpu-seconds 0"
N="python3 bench.py --case netdes --steps 4 --warmup 1 --conv-iters 0 --cpu-seconds 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/hyd -o run -- $H > $O/hyd.log 2>&1
rc=$?; echo "hydro pmc $rc"; [ $rc -eq 0 ] || { tail -5 $O/hyd.log; exit $rc; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/nf -o run -- $N > $O/nf.log 2>&1
rc=$?; echo "netdes fetch $rc"; [ $rc -eq 0 ] || { tail -5 $O/nf.log; exit $rc; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/nw -o run -- $N > $O/nw.log 2>&1
rc=$?; echo "netdes write $rc"; [ $rc -eq 0 ] || { tail -5 $O/nw.log; exit $rc; }
python3 tools/traffic_from_pmc.py $O/nf/run_counter_collection.csv $O/nw/run_counter_collection.csv block $O/netdes_traffic.json netdes "--case netdes" && cat $O/netdes_traffic.json | head -14
grep '^{"metric' $O/nf.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print('netdes', d['ms_per_step'], r.get('pdhg_iters_per_scen_per_step'), d['config'].get('scenarios'))"
