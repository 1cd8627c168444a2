# Round 3: PMC bytes (FETCH / WRITE passes) of the final netdes and sslp kernels, and their bench lines
# with those bytes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ap
rm -rf $O; mkdir -p $O
for c in "netdes --scen 1024" "sslp --scen 4096"; do
  n=$(echo $c | cut -d' ' -f1)
  B="bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case $c"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$n/fetch -o run -- python3 $B > $O/$n.fetch.log 2>&1 || { echo "$n fetch failed"; tail -3 $O/$n.fetch.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$n/write -o run -- python3 $B > $O/$n.write.log 2>&1 || { echo "$n write failed"; tail -3 $O/$n.write.log; exit 1; }
  python3 tools/traffic_from_pmc.py $O/$n/fetch/run_counter_collection.csv $O/$n/write/run_counter_collection.csv block $O/${n}_traffic.json $n "--case $c" > /dev/null || exit 1
  timeout -k 10 300 python3 -u $B --traffic-json $O/${n}_traffic.json > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), r.get('hbm_measured_GBs'), r.get('hbm_measured_frac'))"
done
