set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ao
mkdir -p $O
for c in "netdes --scen 1024" "farmer"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case $c > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], json.dumps(d['roofline'])[:400])"
done
