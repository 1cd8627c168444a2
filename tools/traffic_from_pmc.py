"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs).

Per /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): both counters are in KB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it is doubled.
The first dispatch of each kernel (PH iteration 0's cold solve / setup) is excluded.

Usage: python tools/traffic_from_pmc.py FETCH_CSV WRITE_CSV LAYOUT OUT_JSON [CASE [BENCH_ARGS]]
"""
import csv
import json
import re
import sys

KERNELS = {"local": r"pdhg_local_kernel", "gather": r"pdhg_kernel<", "block": r"pdhg_block_kernel",
           "mfma": r"pdhg_mfma_kernel", "stream": r"pdhg_stream_kernel", "border": r"pdhg_border(_reg)?_kernel",
           "wave": r"pdhg_wave_kernel"}
AUX = {"node_sums": r"node_sums_kernel", "w_update": r"w_update_kernel", "xbar_head": r"xbar_head_kernel"}


def per_launch_kb(path, pattern, counter):
    vals, name = [], None
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and re.search(pattern, r["Kernel_Name"]):
            vals.append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]
    vals = vals[1:] if len(vals) > 1 else vals
    return (sum(vals) / len(vals) if vals else None), len(vals), name


def main(fetch_csv, write_csv, layout, out, case="farmer", args=""):
    pat = KERNELS[layout]
    f_kb, nf, name = per_launch_kb(fetch_csv, pat, "FETCH_SIZE")
    w_kb, nw, _ = per_launch_kb(write_csv, pat, "WRITE_SIZE")
    res = {"case": case, "bench_args": args, "layout": layout, "pdhg_kernel": name, "launches": [nf, nw],
           "pdhg_fetch_kb_raw": f_kb, "pdhg_write_kb": w_kb,
           "pdhg_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024) if f_kb is not None else None}
    for k, p in AUX.items():
        fk, _, _ = per_launch_kb(fetch_csv, p, "FETCH_SIZE")
        wk, _, _ = per_launch_kb(write_csv, p, "WRITE_SIZE")
        res[f"{k}_bytes_per_launch"] = int(2 * fk * 1024 + wk * 1024) if fk is not None and wk is not None else None
    res["method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                     "the `bench.py` workload named by case / bench_args; KB units; FETCH doubled (gfx950 correction, "
                     "MI355X_MICROARCH.md); per PH-iteration launch, first dispatch excluded")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:7])
