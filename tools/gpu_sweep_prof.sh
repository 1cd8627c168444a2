# PH-update sweep at S*N = 1e8 with its kernel trace and FETCH / WRITE PMC passes (separate runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sweep
mkdir -p $O
timeout -k 10 300 python -u tools/ph_update_sweep.py $O/sweep.json > $O/sweep.log 2>&1 || { tail -5 $O/sweep.log; exit 1; }
export SWEEP_CASES=100000x1000
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/ph_update_sweep.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/ph_update_sweep.py > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/ph_update_sweep.py > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
def per(path, counter, pat):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and pat in r["Kernel_Name"]]
    v = v[2:] if len(v) > 2 else v          # the checked first update excluded
    return sum(v) / len(v) if v else None
F = glob.glob("gpurun_out/sweep/fetch/**/*counter_collection.csv", recursive=True)[0]
W = glob.glob("gpurun_out/sweep/write/**/*counter_collection.csv", recursive=True)[0]
out = {}
for k, pat in (("node_sums", "node_sums_kernel"), ("w_update", "w_update_kernel")):
    f, w = per(F, "FETCH_SIZE", pat), per(W, "WRITE_SIZE", pat)
    out[k] = {"fetch_kb_raw": f, "write_kb": w, "bytes": int(2 * f * 1024 + w * 1024) if f and w else None}
out["total_bytes_per_update"] = sum(v["bytes"] for v in out.values() if isinstance(v, dict) and v["bytes"])
out["algorithmic_bytes_per_update"] = 8 * 100000 * 1000 * 4 + 8 * 100000 + 16 * 1000
out["method"] = "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, KB, FETCH doubled (gfx950, MI355X_MICROARCH.md)"
json.dump(out, open("gpurun_out/sweep/traffic.json", "w"), indent=1)
print(json.dumps(out))
PY
