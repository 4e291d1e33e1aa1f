"""Summarise tools/pmc_flops.sh: per config, net_kernel's issued fp64 flops per pair.
On gfx950 SQ_INSTS_VALU_FLOPS_FP64 (+ _FP64_TRANS) counts the flops of each issued fp64
wave-instruction once (FMA = 2), not per lane — it tracks 2·FMA + ADD + MUL within a few
percent — so × 64 it is the flops of every lane of every issued fp64 instruction, idle
lanes included (an upper bound of the useful flops; the 28×28 epilogues fill 112 of 128
lanes).  Over the traced dispatch time of 3 B = 1024 Kxz tiles (1024² pairs each).
Writes <out>/flops_pmc.json."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
res = {}
pairs = 3 * 1024 * 1024
for d in sorted(glob.glob(os.path.join(out, "*_fl"))):
    cfg = os.path.basename(d)[:-3]
    tot = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "net_kernel" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not tot:
        continue
    ns = 0.0
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "net_kernel" in r["Kernel_Name"]:
                ns += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    fl = tot.get("SQ_INSTS_VALU_FLOPS_FP64", 0.0) + tot.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0)
    wave = (2 * tot.get("SQ_INSTS_VALU_FMA_F64", 0.0) + tot.get("SQ_INSTS_VALU_ADD_F64", 0.0) +
            tot.get("SQ_INSTS_VALU_MUL_F64", 0.0) + tot.get("SQ_INSTS_VALU_TRANS_F64", 0.0)) * 64
    res[cfg] = dict(tot)
    issued = 64 * fl
    cyc = 4 * (tot.get("SQ_INSTS_VALU_FMA_F64", 0.0) + tot.get("SQ_INSTS_VALU_ADD_F64", 0.0) +
               tot.get("SQ_INSTS_VALU_MUL_F64", 0.0)) + 16 * tot.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
    res[cfg].update(
        net_kernel_ns=ns,
        issued_lane_flops_per_pair=issued / pairs,
        wave_instruction_flops_per_pair=wave / pairs,
        issued_tflops_under_pmc=(issued / (ns * 1e-9) / 1e12) if ns else None,
        fp64_simd_cycles_per_pair=cyc / pairs,
        trans_share_of_fp64_cycles=(16 * tot.get("SQ_INSTS_VALU_TRANS_F64", 0.0) / cyc) if cyc else None,
        note="sums over the net_kernel dispatches of 3 B=1024 Kxz tiles; issued lane flops = "
             "64 x (SQ_INSTS_VALU_FLOPS_FP64 + SQ_INSTS_VALU_FLOPS_FP64_TRANS) (per-instruction "
             "flop counts on gfx950, FMA = 2; every lane of each issued fp64 instruction); "
             "fp64 SIMD cycles = 4 per FMA/ADD/MUL and 16 per v_rsq_f64 wave-instruction "
             "(measured issue costs, DESIGN.md section 4.1)")
json.dump(res, open(os.path.join(out, "flops_pmc.json"), "w"), indent=1)
print(json.dumps({k: {a: b for a, b in v.items() if a != "note"} for k, v in res.items()},
                 indent=1))
