# Round 3: netdes (unit codes + row segments) VALU / LDS issue counters, one PMC pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ak
rm -rf $O; mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 3 --warmup 1 --conv-iters 0 --cpu-seconds 0 --case netdes --scen 1024 > $O/pmc.log 2>&1
rc=$?; echo "pmc exit $rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc.log; exit 1; }
f=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
    if "pdhg_block" not in k: continue
    agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
ds = sorted(agg, key=int)[1:]   # skip Iter0
tot = collections.defaultdict(float)
for d in ds:
    for c, v in agg[d].items(): tot[c] += v / len(ds)
print({c: f"{v:.4g}" for c, v in tot.items()})
PY
