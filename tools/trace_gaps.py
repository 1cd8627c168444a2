"""Summarise a rocprofv3 kernel trace (its SQLite results database) into the per-step timeline of
the PH loop: kernel durations and the idle gaps between consecutive kernels, by kernel kind.

    python tools/trace_gaps.py gpurun_out/.../run_results.db [--first 12 --count 28] > summary.json

`--first` / `--count` select PDHG solve launches by position (skip Iter0 and the warmup)."""
import argparse
import json
import sqlite3
import statistics


def kind(name):
    for key, k in (("pdhg_local", "solve"), ("pdhg_block", "solve"), ("node_sums", "node_sums"),
                   ("schedule", "schedule"), ("w_update", "w_update"), ("xbar_head", "xbar_head")):
        if key in name:
            return k
    return name.split("(")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first", type=int, default=12)
    ap.add_argument("--count", type=int, default=28)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, start, end from kernels order by start").fetchall()
    solves = [i for i, r in enumerate(rows) if kind(r[0]) == "solve"][a.first:a.first + a.count]
    lo, hi = solves[0], solves[-1]
    dur, gap = {}, {}
    for i in range(lo, hi):
        k = kind(rows[i][0])
        dur.setdefault(k, []).append((rows[i][2] - rows[i][1]) / 1e3)
        nxt = kind(rows[i + 1][0])
        gap.setdefault(f"{k}->{nxt}", []).append((rows[i + 1][1] - rows[i][2]) / 1e3)
    starts = [rows[i][1] for i in solves]
    out = {"solves": len(solves),
           "period_us_median": statistics.median([(b - a_) / 1e3 for a_, b in zip(starts, starts[1:])]),
           "duration_us_median": {k: round(statistics.median(v), 2) for k, v in dur.items()},
           "gap_us_median": {k: round(statistics.median(v), 2) for k, v in gap.items()},
           "counts": {k: len(v) for k, v in dur.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
