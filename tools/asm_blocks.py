"""Instruction counts of a kernel's PDHG inner loop and of the basic blocks after it (the
restart / termination check), from `hipcc --cuda-device-only -S` output.

Usage: python tools/asm_blocks.py ASM_FILE MANGLED_KERNEL_NAME
"""
import sys
from collections import Counter


def isins(l):
    t = l.strip()
    return t and not t.startswith((";", ".", "//"))


def main(path, name):
    s = open(path).read()
    i = s.index(name + ":")
    body = s[i:s.index(".Lfunc_end", i)].splitlines()
    hdr = [k for k, l in enumerate(body) if "Inner Loop Header" in l][0]
    lab = body[hdr - 1].split(":")[0].strip()
    end = [k for k, l in enumerate(body) if lab in l and "cbranch" in l][0]
    inner = [l for l in body[hdr:end + 1] if isins(l)]
    print("inner loop:", len(inner), Counter(l.split()[0] for l in inner).most_common(8))
    cur = None
    blocks = []
    for l in body[end + 1:]:
        t = l.strip()
        if t.startswith(".LBB"):
            cur = [t.split(":")[0], 0, 0, ""]
            blocks.append(cur)
            continue
        if cur is None:
            cur = ["(fall)", 0, 0, ""]
            blocks.append(cur)
        if isins(l):
            cur[1] += 1
            cur[2] += "readlane" in t or "writelane" in t
            if "branch" in t:
                cur[3] = t
    for b in blocks:
        print(f"{b[0]:12s} {b[1]:5d} lane-ops {b[2]:3d}  {b[3]}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
