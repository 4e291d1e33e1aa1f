"""Summarise tools/pmc_valu_mix.sh: per (variant, config) and net_kernel stage, VALU
wave-instructions per pair by class — fp64 arithmetic (FMA + ADD + MUL + TRANS), 32-bit
and 64-bit integer, conversions, and the rest (moves, selects, fp64 max / compares, lane
transfers) — over 3 B = 1024 Kxz tiles (3·1024² pairs).  Writes <out>/valu_mix.json."""
import collections
import csv
import glob
import json
import os
import re
import sys

out = sys.argv[1]
pairs = 3 * 1024 * 1024
res = {}
for d in sorted(glob.glob(os.path.join(out, "*_*"))):
    if not os.path.isdir(d):
        continue
    tag = os.path.basename(d)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "net_kernel" not in name:
                continue
            m = re.search(r"net_kernel<[^>]*?(-?\d+)>", name)
            stage = m.group(1) if m else name[:60]
            per[stage][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        continue
    rows = {}
    tot = collections.defaultdict(float)
    for stage, c in per.items():
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64",
                                           "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
        v = c.get("SQ_INSTS_VALU", 0.0)
        i32, i64, cvt = (c.get("SQ_INSTS_VALU_INT32", 0.0), c.get("SQ_INSTS_VALU_INT64", 0.0),
                         c.get("SQ_INSTS_VALU_CVT", 0.0))
        row = {"valu": v / pairs, "fp64_arith": f64 / pairs, "int32": i32 / pairs,
               "int64": i64 / pairs, "cvt": cvt / pairs,
               "rest": (v - f64 - i32 - i64 - cvt) / pairs}
        rows[f"program {stage}"] = {k: round(x, 1) for k, x in row.items()}
        for k, x in row.items():
            tot[k] += x
    rows["total"] = {k: round(x, 1) for k, x in tot.items()}
    res[tag] = rows
json.dump(res, open(os.path.join(out, "valu_mix.json"), "w"), indent=1)
for tag, rows in res.items():
    print(tag, json.dumps(rows["total"]))
