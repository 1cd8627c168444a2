# round 6: the per-lane-atomic schedule (256 threads, 4 rows in flight) fused into the node-sum head at 10k
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_q; mkdir -p $O
p() {  # tag env scen
  tag=$1; envv=$2; sc=$3
  env $envv timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 bench.py --scen $sc --steps 40 --warmup 5 --conv-iters 0 --cpu-seconds 0 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  python3 - "$O/$tag/run_kernel_stats.csv" "$tag" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "node_sums_kernel<false, true>" in r["Name"] or "schedule_kernel" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], "calls", r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 2), "max", round(float(r["MaxNs"]) / 1e3, 2))
PY
}
b() {  # tag env bench-args
  tag=$1; shift; envv=$1; shift
  env $envv timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); t=d.get('time_to_conv',{}); r=d['roofline']
print('$tag', d['ms_per_step'], r.get('avg_launch_ms'), d.get('host_and_exchange_ms_per_step'), t.get('seconds'), t.get('ph_iters'))"
}
p f1 PHG_SCHED_FUSE=1 10000
p f0 PHG_SCHED_FUSE=0 10000
for rep in 1 2; do
  b fuse1_$rep PHG_SCHED_FUSE=1
  b fuse0_$rep PHG_SCHED_FUSE=0
done
