# find the first stalling solve of the farmer 10k trajectory, then replay up to it with the PROF
# kernel printing that scenario's every check (PHG_WATCH_SCEN)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/stall; mkdir -p $O
STALL_STOP=1 timeout -k 10 400 python -u tools/stall/find_stall.py > $O/find.log 2>&1 || { tail -5 $O/find.log; exit 1; }
tail -4 $O/find.log
line=$(grep "^STALL" $O/find.log) || { echo "no stall found"; exit 0; }
k=$(echo $line | cut -d' ' -f2); s=$(echo $line | cut -d' ' -f3)
STALL_K=$k PHG_LOCAL_PROF=1 PHG_WATCH_SCEN=$s timeout -k 10 400 python -u tools/stall/find_stall.py > $O/watch.log 2>&1 || { tail -5 $O/watch.log; exit 1; }
grep -c PHG_WATCH $O/watch.log; grep "^step" $O/watch.log | tail -2
