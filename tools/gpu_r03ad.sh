# Round 3: rocprofv3 kernel-trace stats of the secondary cases on their round-3 kernels (sslp row
# segments, netdes unit codes + segments, UC at the size-based theta with plain launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ad
rm -rf $O; mkdir -p $O
for c in "sslp --scen 4096" "netdes --scen 1024" "uc"; do
  n=$(echo $c | cut -d' ' -f1)
  PHG_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case $c > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rocprofv3 exit $rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
  f=$(find $O/$n -name "*kernel_stats.csv" | head -1); head -4 "$f" | cut -c1-220
done
