"""PMC bytes of the folded PH update (tools/ph_update_sweep.py run_fold under separate FETCH_SIZE /
WRITE_SIZE rocprofv3 passes): per dispatch of the PDHG solve with the fold and without, their
difference (the prologue's W update), plus the node-sum and x-bar-head launches of the folded
iteration.  FETCH_SIZE doubled (gfx950 correction, MI355X_MICROARCH.md).

Usage: python tools/fold_traffic.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import glob
import json
import sys


def series(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in rows]


def main(fd, wd, out):
    res = {}
    for counter, d, scale in (("FETCH_SIZE", fd, 2.0), ("WRITE_SIZE", wd, 1.0)):
        s = series(d, counter)
        pd = [v * scale * 1024 for k, v in s if "pdhg_local_kernel" in k]
        ns = [v * scale * 1024 for k, v in s if "node_sums_kernel" in k]
        hd = [v * scale * 1024 for k, v in s if "xbar_head_kernel" in k]
        # run_fold: one warm solve, then per tag (fold, nofold): 1 + reps solves (reps = 10)
        reps = 10
        fold = pd[2:1 + 1 + reps]          # the fold tag's timed solves (after its first)
        nofold = pd[1 + 1 + reps + 1:]     # the nofold tag's timed solves
        res[counter] = {"solve_fold": sum(fold) / len(fold), "solve_nofold": sum(nofold) / len(nofold),
                        "node_sums": sum(ns) / len(ns) if ns else None, "xbar_head": sum(hd) / len(hd) if hd else 0.0}
    F, W = res["FETCH_SIZE"], res["WRITE_SIZE"]
    prologue = (F["solve_fold"] - F["solve_nofold"]) + (W["solve_fold"] - W["solve_nofold"])
    upd = F["node_sums"] + W["node_sums"] + F["xbar_head"] + W["xbar_head"]
    S, N = 1000000, 100
    alg = 8 * S * N * 3 + 8 * S + 16 * N
    out_d = {"S": S, "N": N, "bytes_node_sums_plus_head": int(upd), "bytes_prologue_extra": int(prologue),
             "bytes_folded_update": int(upd + prologue), "algorithmic_3_stream_bytes": alg,
             "ratio_to_algorithmic": round((upd + prologue) / alg, 4), "per_counter": res,
             "method": __doc__.split("\n\n")[0]}
    json.dump(out_d, open(out, "w"), indent=1)
    print(json.dumps(out_d))


if __name__ == "__main__":
    main(*sys.argv[1:4])
