# round 6: node-sum head (HEADX) duration by final-rank width / segment count, kernel trace per config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_j; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loop.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
p() {  # tag env scen
  tag=$1; envv=$2; sc=$3
  env $envv timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 bench.py --scen $sc --steps 40 --warmup 5 --conv-iters 0 --cpu-seconds 0 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  python3 - "$O/$tag/run_kernel_stats.csv" "$tag" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "node_sums_kernel<false, true>" in r["Name"]:
        print(sys.argv[2], "HEADX avg us", round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2))
PY
}
for sc in 10000 1250; do
  p s${sc}_def X=0 $sc
  p s${sc}_f1024 PHG_NFINAL_LOADS=1024 $sc
  p s${sc}_f512 PHG_NFINAL_LOADS=512 $sc
  p s${sc}_f4096 PHG_NFINAL_LOADS=4096 $sc
  p s${sc}_seg128 PHG_NODESEG_MAX=128 $sc
  p s${sc}_seg64 PHG_NODESEG_MAX=64 $sc
  p s${sc}_seg512 PHG_NODESEG_MAX=512 $sc
done
