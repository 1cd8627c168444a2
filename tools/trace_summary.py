"""Timed-region launch durations from a rocprofv3 kernel trace (``*_kernel_trace.csv``).

rocprofv3's --stats average covers every dispatch of a kernel, including PH iteration 0's cold
solve, the warmup iterations and the extra iterations bench.py runs after the timed region (the
PH-update timing); bench.py's HIP-event average covers the STEPS timed dispatches of the PDHG
kernel, which follow Iter0 and WARMUP warmup dispatches.  This prints both ("avg_ms_timed": the
dispatches [1 + WARMUP, 1 + WARMUP + STEPS)), so the two can be compared like for like.

Usage: python tools/trace_summary.py TRACE_CSV STEPS OUT_JSON [WARMUP]
"""
import csv
import json
import re
import sys

PATS = {"pdhg": r"pdhg_(local_|block_)?kernel", "node_sums": r"node_sums_kernel",
        "w_update": r"w_update_kernel", "schedule": r"schedule_kernel"}


def main(trace, steps, out, warmup=5):
    steps, skip = int(steps), 1 + int(warmup)
    rows = list(csv.DictReader(open(trace)))
    res = {"trace": trace, "steps": steps}
    for k, p in PATS.items():
        sel = [r for r in rows if re.search(p, r["Kernel_Name"])]
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
        if not d:
            continue
        res[k] = {"kernel": sel[0]["Kernel_Name"], "dispatches": len(d),
                  "avg_ms_all": round(sum(d) / len(d), 5),
                  "avg_ms_last_steps": round(sum(d[-steps:]) / len(d[-steps:]), 5)}
        if k == "pdhg" and len(d) >= skip + steps:
            res[k]["avg_ms_timed"] = round(sum(d[skip:skip + steps]) / steps, 5)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
