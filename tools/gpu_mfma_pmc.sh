# MFMA counters of the shared-matrix kernel on hydro at full occupancy (100 000 scenarios): one
# rocprofv3 --pmc pass (SQ counters only), summarised per launch like profiles/pmc_r02/summary.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_h100k
mkdir -p $O
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O -o run -- python3 bench.py --steps 5 --warmup 2 --conv-iters 0 --cpu-seconds 0 --case hydro --scen 100000 > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
from collections import defaultdict
f = glob.glob("gpurun_out/pmc_h100k/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(dict)
name = None
for r in csv.DictReader(open(f)):
    if "pdhg_mfma_kernel" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        per[r["Dispatch_Id"]]["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name = r["Kernel_Name"]
ds = sorted(per, key=int)[1:]          # the first (Iter0) dispatch excluded
avg = {k: sum(per[d][k] for d in ds) / len(ds) for k in per[ds[0]]}
avg["kernel"] = name
avg["clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / avg["dur_ms"] / 1e6   # GRBM summed over the 8 XCDs
avg["mfma_busy_frac_of_simd_cycles"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] * 128)
avg["workload"] = "hydro 3-stage tree, 100 000 scenarios, MFMA layout (bench.py --case hydro --scen 100000)"
json.dump(avg, open("gpurun_out/pmc_h100k/summary.json", "w"), indent=1)
print(json.dumps(avg))
PY
