set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/hstall; mkdir -p $O
STALL_THETA=${STALL_THETA:-0.5} timeout -k 10 300 python -u tools/stall/hydro_stall.py > $O/find.log 2>&1 || { tail -5 $O/find.log; exit 1; }
cat $O/find.log | grep -v amdgpu.ids
s=$(grep "^STALL" $O/find.log | head -1 | cut -d' ' -f2)
[ -n "$s" ] || exit 0
STALL_THETA=${STALL_THETA:-0.5} PHG_WATCH_SCEN=$s timeout -k 10 300 python -u tools/stall/hydro_stall.py > $O/watch.log 2>&1 || { tail -5 $O/watch.log; exit 1; }
grep -c PHG_WATCH $O/watch.log
