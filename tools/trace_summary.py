"""Timed-region launch durations from a rocprofv3 kernel trace (``*_kernel_trace.csv``).

rocprofv3's --stats average covers every dispatch of a kernel, including PH iteration 0's cold
solve and the warmup iterations; bench.py's HIP-event average covers only the last STEPS
dispatches of the PDHG kernel.  This prints both, so the two can be compared like for like.

Usage: python tools/trace_summary.py TRACE_CSV STEPS OUT_JSON
"""
import csv
import json
import re
import sys

PATS = {"pdhg": r"pdhg_(local_|block_)?kernel", "node_sums": r"node_sums_kernel",
        "w_update": r"w_update_kernel", "schedule": r"schedule_kernel"}


def main(trace, steps, out):
    steps = int(steps)
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
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
