"""Executed fp64 operations per PDHG iteration in the lane-local kernel's hot loop: the compiled
inner loop (hipcc --cuda-device-only -S, two PDHG iterations per trip) against
pdhg_local.hip local_loop_ops (restated here line for line).

Usage: python tools/loop_ops.py [ASM_FILE]   (default: compiles pdhg_local.hip to /tmp)
Prints one JSON line per pattern-specialised farmer variant: ISA counts per lane per PDHG
iteration (FMA = 2, add / mul / max / min = 1) and the local_loop_ops value."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FARMER_BI = (1 << 18) | (1 << 19) | (1 << 40) | (1 << 33) | (1 << 48)
FARMER_BF = 0x2010003000f


def loop_ops(LPS, CPL, RPL, D, MB, MC, BI, BF):
    FOLD = RPL * CPL + D * CPL <= 12
    FOLDT = FOLD and (bin(MB).count("1") + bin(MC).count("1") <= 8)
    bon = lambda r, k: (MB >> (r * CPL + k)) & 1
    con = lambda d, k: (MC >> (d * CPL + k)) & 1
    inf = lambda b: (BI >> b) & 1
    finb = lambda b: (BF >> b) & 1
    ops = 0
    for k in range(CPL):
        e = sum(bon(r, k) for r in range(RPL)) + sum(con(d, k) for d in range(D))
        ops += 2 * (2 + 2 * e) if FOLDT else 2 * 4
        ops += 2 * ((0 if inf(k) else 1) + (0 if inf(16 + k) else 1))
        if not FOLDT:
            ops += 2 * (2 * e - 1 if e else 0)
        ops += 1
    for r in range(RPL):
        e = sum(bon(r, k) for k in range(CPL))
        one = (finb(32 + r) and inf(40 + r)) or (finb(40 + r) and inf(32 + r))
        ops += 2 * (2 * e if one else (2 * e - 1 if e else 0))
        ops += 2 * (5 if one else 4 + (0 if inf(32 + r) else 1) + (0 if inf(40 + r) else 1) + 1)
        ops += 1
    lg = LPS.bit_length() - 1
    for d in range(D):
        e = sum(con(d, k) for k in range(CPL))
        one = (finb(48 + d) and inf(52 + d)) or (finb(52 + d) and inf(48 + d))
        ops += 2 * ((2 * e if one else (2 * e - 1 if e else 0)) + lg)
        ops += 2 * (5 if one else 4 + (0 if inf(48 + d) else 1) + (0 if inf(52 + d) else 1) + 1)
        ops += 1
    return ops * 50


def isa_counts(asm, name):
    i = asm.index(name + ":")
    body = asm[i:asm.index(".Lfunc_end", i)].splitlines()
    hdr = [k for k, l in enumerate(body) if "Inner Loop Header" in l][0]
    lab = body[hdr - 1].split(":")[0].strip()
    end = [k for k, l in enumerate(body) if lab in l and "cbranch" in l][0]
    ins = [l.split()[0] for l in body[hdr:end + 1] if l.strip() and not l.strip().startswith((";", ".", "//"))]
    fma = sum(op.startswith(("v_fma_f64", "v_fmac_f64")) for op in ins)
    one = sum(op.startswith(("v_add_f64", "v_mul_f64", "v_max_f64", "v_min_f64")) for op in ins)
    return {"instructions": len(ins), "fp64_fma": fma, "fp64_other": one, "ops_per_2_iters": 2 * fma + one}


def main():
    if len(sys.argv) > 1:
        asm = open(sys.argv[1]).read()
    else:
        out = "/tmp/pdhg_local_loop_ops.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        os.path.join(ROOT, "mpi-sppy_amd", "csrc", "pdhg_local.hip"), "-o", out], check=True)
        asm = open(out).read()
    for bf, tag in ((FARMER_BF, ""), (FARMER_BF | (1 << 52), " free")):
        for lps in (16, 32, 64):
            for wv in (2, 1):
                name = (f"_ZN3phg17pdhg_local_kernelILi{lps}ELi4ELi2ELi1ELb0ELj127ELj1ELy{FARMER_BI}ELy{bf}ELj1ELi{wv}EEEvNS_8PdhgArgsE")
                if name + ":" not in asm:
                    continue
                c = isa_counts(asm, name)
                want = loop_ops(lps, 4, 2, 1, 0x7F, 0x1, FARMER_BI, bf)
                print(json.dumps({"variant": f"farmer{tag} LPS={lps} WV={wv}", **c,
                                  "isa_ops_per_lane_iter": c["ops_per_2_iters"] / 2,
                                  "local_loop_ops_per_lane_iter": want / 100}))


if __name__ == "__main__":
    main()
