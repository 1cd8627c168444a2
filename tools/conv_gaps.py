"""Where the time-to-conv run's wall time goes: from a rocprofv3 kernel trace of
`bench.py` (its conv run is the trace's last stretch of PDHG launches), sum the device time per
kernel over the last K PH iterations and the idle gaps between consecutive kernels.

Usage: python tools/conv_gaps.py TRACE_DIR [K]"""
import csv
import os
import sys
from collections import defaultdict


def main(d, k=5000):
    k = int(k)
    ev = []
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if "pdhg" in e[2]]
    i0 = idx[-k]
    sel = ev[i0:]
    span = (sel[-1][1] - sel[0][0]) / 1e3
    per = defaultdict(lambda: [0, 0.0])
    gaps = 0.0
    big = 0
    prev = None
    for s, e, nm in sel:
        per[nm][0] += 1
        per[nm][1] += (e - s) / 1e3
        if prev is not None and s > prev:
            gaps += (s - prev) / 1e3
            big += (s - prev) > 20000
        prev = max(prev or 0, e)
    print(f"last {k} PH iterations: span {span / 1e3:.3f} ms... per iteration {span / k:.2f} us")
    for nm, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {nm:48s} {c:6d} launches {t / 1e3:9.3f} ms  {t / k:8.2f} us/iter")
    print(f"  idle gaps {gaps / 1e3:9.3f} ms  {gaps / k:8.2f} us/iter ({big} gaps > 20 us)")


if __name__ == "__main__":
    main(*sys.argv[1:])
