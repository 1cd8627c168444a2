"""VALU instruction mix of the headline kernel: the two rocprofv3 --pmc passes of
tools/gpu_pmc_mix.sh (SQ_INSTS_VALU and its class counters, per dispatch) beside the compiled hot
loop's instruction histogram (tools/loop_ops.py's ISA parse), and an issue model priced by
MI355X_MICROARCH.md: a wave64 fp64 VALU instruction occupies its SIMD 4 cycles (16 fp64 FMA lanes
per cycle: 78.6 TFLOP/s = 1 024 SIMDs x 32 flop x 2.4 GHz), a 32-bit one 2 cycles (row
'v_fma_f32 (wave64)', line 473: two waves per SIMD, as this kernel runs).

Usage: python tools/pmc_mix.py [PMC_DIR] [OUT_JSON]
  PMC_DIR  default gpurun_out/pmc_mix (p1/, p2/ run_counter_collection.csv)
  OUT_JSON default profiles/r06/pmc_valu_mix.json
"""
import collections
import csv
import json
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import loop_ops  # noqa: E402

KERNEL = "pdhg_local_kernel<32, 4, 2, 1, false, 127u, 1u"
# the variant PH's solves run (free nonants: the coupling row's finite side compiled in, round 6)
SYMBOL = (f"_ZN3phg17pdhg_local_kernelILi32ELi4ELi2ELi1ELb0ELj127ELj1ELy{loop_ops.FARMER_BI}"
          f"ELy{loop_ops.FARMER_BF | (1 << 52)}ELj1ELi2EEEvNS_8PdhgArgsE")
F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64")


def dispatches(pmc_dir):
    """{dispatch id: {counter: value}} of the headline kernel over both passes' CSVs (one dict per
    pass: the passes are separate runs, their dispatch ids line up by order)."""
    per_pass = []
    for p in ("p1", "p2"):
        d = collections.defaultdict(dict)
        for r in csv.DictReader(open(os.path.join(pmc_dir, p, "run_counter_collection.csv"))):
            if KERNEL in r["Kernel_Name"]:
                d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
                d[int(r["Dispatch_Id"])]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per_pass.append([d[k] for k in sorted(d)])
    return per_pass


def steady(rows):
    """the PH-iteration launches: drop the Iter0 LP solve (and anything > 2x the median count)"""
    key = "SQ_INSTS_VALU" if "SQ_INSTS_VALU" in rows[0] else "SQ_ACTIVE_INST_VALU"
    med = statistics.median(r[key] for r in rows)
    return [r for r in rows if r[key] <= 2 * med]


def isa_histogram():
    out = "/tmp/pdhg_local_mix.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    os.path.join(ROOT, "mpi-sppy_amd", "csrc", "pdhg_local.hip"), "-o", out], check=True)
    asm = open(out).read()
    i = asm.index(SYMBOL + ":")
    body = asm[i:asm.index(".Lfunc_end", i)].splitlines()
    hdr = [k for k, l in enumerate(body) if "Inner Loop Header" in l][0]
    lab = body[hdr - 1].split(":")[0].strip()
    end = [k for k, l in enumerate(body) if lab in l and "cbranch" in l][0]
    lines = [l.strip() for l in body[hdr:end + 1] if l.strip() and not l.strip().startswith((";", ".", "//"))]
    cls = collections.Counter()
    for l in lines:
        op = l.split()[0]
        if op.startswith(("v_fma_f64", "v_fmac_f64")):
            c = "fp64 fma"
        elif op.startswith(("v_add_f64", "v_mul_f64")):
            c = "fp64 add/mul"
        elif op.startswith(("v_max_f64", "v_min_f64")):
            c = "fp64 max/min"
        elif op.startswith("v_mov_b32") and ("row_" in l or "quad_perm" in l or "row_ror" in l):
            c = "32-bit DPP move (group sums)"
        elif op.startswith(("v_permlane", "v_mov_b32_dpp")):
            c = "32-bit permlane swap (group sums)"
        elif op.startswith("v_cndmask"):
            c = "32-bit select"
        elif op.startswith("v_"):
            c = "other VALU (" + re.sub(r"_e(32|64)$", "", op) + ")"
        elif op.startswith("s_"):
            c = "scalar / branch / wait"
        else:
            c = "other"
        cls[c] += 1
    return {"instructions_per_2_iterations": len(lines), "by_class": dict(cls.most_common())}


def main():
    pmc_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_mix")
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r06", "pmc_valu_mix.json")
    p1, p2 = (steady(r) for r in dispatches(pmc_dir))
    avg = {}
    for rows in (p1, p2):
        for c in rows[0]:
            if c != "_ns":
                avg[c] = statistics.fmean(r[c] for r in rows)
    waves = avg["SQ_WAVES"]
    per_wave = {c: v / waves for c, v in avg.items() if c.startswith("SQ_INSTS")}
    valu = per_wave["SQ_INSTS_VALU"]
    f64 = sum(per_wave.get(c, 0.0) for c in F64)
    rest32 = valu - f64 - per_wave.get("SQ_INSTS_VALU_INT64", 0.0)
    # ISA: per PDHG iteration of the hot loop
    isa = isa_histogram()
    h = isa["by_class"]
    it_f64_fma = h.get("fp64 fma", 0) / 2
    it_f64_other = (h.get("fp64 add/mul", 0) + h.get("fp64 max/min", 0)) / 2
    it_valu = sum(v for k, v in h.items() if not k.startswith(("scalar", "other ("))) / 2
    # wave-iterations per launch: the hot loop's fp64 FMAs per iteration divide the counted FMAs
    # (the checks / prologue / epilogue FMAs are few by comparison; quoted as an upper bound)
    wave_iters = per_wave["SQ_INSTS_VALU_FMA_F64"] / it_f64_fma
    # issue model (cycles one SIMD spends issuing one wave's instructions)
    cyc_f64 = 4.0 * (f64 + per_wave.get("SQ_INSTS_VALU_INT64", 0.0))
    cyc_32 = 2.0 * rest32
    # max / min f64 are not in the F64 class counters (the ISA has them; see isa_check): priced
    # at 4 like every fp64 instruction, they move from the 32-bit remainder
    maxmin = (h.get("fp64 max/min", 0) / 2) * wave_iters
    cyc_model = cyc_f64 + cyc_32 + 2.0 * maxmin
    ns = statistics.fmean(r["_ns"] for r in p1)
    clock = avg["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9)
    simds = 1024
    waves_per_simd = waves / simds
    simd_cycles = ns * 1e-9 * clock
    res = {
        "kernel": "pdhg_local_kernel<32,4,2,1> farmer pattern build (farmer cm=10, 10 000 scenarios, two waves per SIMD)",
        "method": "rocprofv3 --pmc, two passes (8 SQ + GRBM_GUI_ACTIVE each) of bench.py --steps 10 --warmup 3 "
                  "--conv-iters 0 (tools/gpu_pmc_mix.sh); the Iter0 LP launch dropped; counters averaged over the "
                  "PH-iteration launches; ISA of the same build (tools/pmc_mix.py)",
        "dispatches_averaged": [len(p1), len(p2)],
        "counters_per_dispatch": avg,
        "per_wave": {"valu": valu, "fp64_fma": per_wave["SQ_INSTS_VALU_FMA_F64"],
                     "fp64_add": per_wave["SQ_INSTS_VALU_ADD_F64"], "fp64_mul": per_wave["SQ_INSTS_VALU_MUL_F64"],
                     "fp64_trans": per_wave["SQ_INSTS_VALU_TRANS_F64"], "int64": per_wave.get("SQ_INSTS_VALU_INT64"),
                     "int32": per_wave["SQ_INSTS_VALU_INT32"], "cvt": per_wave["SQ_INSTS_VALU_CVT"],
                     "f32": per_wave["SQ_INSTS_VALU_ADD_F32"] + per_wave["SQ_INSTS_VALU_MUL_F32"]
                     + per_wave["SQ_INSTS_VALU_FMA_F32"],
                     "unclassified_32bit (dpp / permlane moves, selects, max/min f64)": valu - f64
                     - per_wave["SQ_INSTS_VALU_INT32"] - per_wave["SQ_INSTS_VALU_CVT"]
                     - per_wave.get("SQ_INSTS_VALU_INT64", 0.0),
                     "salu": per_wave["SQ_INSTS_SALU"], "lds": per_wave["SQ_INSTS_LDS"], "vmem": per_wave["SQ_INSTS_VMEM"]},
        "shares_of_valu": {"fp64 (fma/add/mul/trans)": f64 / valu, "fp64 fma": per_wave["SQ_INSTS_VALU_FMA_F64"] / valu,
                           "everything else": 1 - f64 / valu},
        "isa_hot_loop": isa,
        "isa_per_pdhg_iteration": {"valu": it_valu, "fp64_fma": it_f64_fma, "fp64_add_mul_max_min": it_f64_other},
        "wave_iterations_per_launch_est": wave_iters,
        "valu_per_wave_iteration_counted": valu / wave_iters,
        "issue_model": {
            "rule": "fp64 wave64 instruction 4 SIMD cycles, 32-bit 2 (MI355X_MICROARCH.md:54, 473); max/min f64 "
                    "from the ISA count",
            "cycles_per_wave": cyc_model,
            "fp64_cycles_share": (cyc_f64 + 4.0 * maxmin) / cyc_model,
            "waves_per_simd": waves_per_simd,
            "modelled_issue_cycles_per_simd": cyc_model * waves_per_simd,
            "measured_cycles_per_launch": simd_cycles,
            "issue_utilisation": cyc_model * waves_per_simd / simd_cycles,
            "clock_GHz_from_GRBM": clock / 1e9,
            "launch_us_profiled": ns / 1e3,
        },
    }
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("per_wave", "shares_of_valu", "isa_per_pdhg_iteration",
                                           "valu_per_wave_iteration_counted", "issue_model")}, indent=1))


if __name__ == "__main__":
    main()
