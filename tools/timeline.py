"""Kernel / copy timeline of the last few PH iterations from a rocprofv3 trace directory."""
import csv
import os
import sys


def main(d, n=30):
    ev = []
    for f in os.listdir(d):
        if f.endswith("kernel_trace.csv"):
            for r in csv.DictReader(open(os.path.join(d, f))):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:44]))
        if f.endswith("memory_copy_trace.csv"):
            for r in csv.DictReader(open(os.path.join(d, f))):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
    ev.sort()
    idx = [i for i, e in enumerate(ev) if "pdhg" in e[2]]
    i0 = idx[-6]
    t0 = ev[i0][0]
    prev = None
    for s, e, nm in ev[i0:i0 + int(n)]:
        gap = (s - prev) / 1000 if prev else 0.0
        print(f"{(s - t0) / 1000:9.1f}us dur {(e - s) / 1000:8.1f} gap {gap:7.1f}  {nm}")
        prev = max(prev or 0, e)


if __name__ == "__main__":
    main(*sys.argv[1:])
