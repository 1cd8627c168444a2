# round 6: node-sum head duration, final-rank loads 1024 vs 2048, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_l; mkdir -p $O
p() {  # tag env scen
  tag=$1; envv=$2; sc=$3
  env $envv timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 bench.py --scen $sc --steps 60 --warmup 5 --conv-iters 0 --cpu-seconds 0 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  python3 - "$O/$tag/run_kernel_stats.csv" "$tag" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "node_sums_kernel<false, true>" in r["Name"]:
        print(sys.argv[2], "HEADX avg us", round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2))
PY
}
for rep in 1 2 3; do
  p f1024_$rep PHG_NFINAL_LOADS=1024 10000
  p f2048_$rep PHG_NFINAL_LOADS=2048 10000
done
