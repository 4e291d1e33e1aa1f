"""Summarise tools/pmc_stage.sh per config and net_kernel program (stage): the wave-cycle
split — parked (SQ_WAIT_ANY: s_waitcnt or s_barrier), issue-stalled (SQ_WAIT_INST_ANY),
issuing (SQ_ACTIVE_INST_ANY) — VALU issue per wave-cycle, the lane fill of the VALU
instructions (SQ_THREAD_CYCLES_VALU / (64 · SQ_ACTIVE_INST_VALU)), the LDS issue stalls,
and each program's share of the kernel time (from the kernel trace).  Writes
<out>/stage_pmc.json."""
import collections
import csv
import glob
import json
import os
import re
import sys

out = sys.argv[1]
res = {}


def prog(name):
    m = re.search(r"net_kernel<[^>]*?(-?\d+)>", name)
    return f"program {m.group(1)}" if m else name[:60]


for d in sorted(glob.glob(os.path.join(out, "*_st"))):
    cfg = os.path.basename(d)[:-3]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "net_kernel" in r.get("Kernel_Name", ""):
                per[prog(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ns = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "net_kernel" in r["Kernel_Name"]:
                ns[prog(r["Kernel_Name"])] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    if not per:
        continue
    tot_ns = sum(ns.values()) or 1.0
    rows = {}
    for p, c in sorted(per.items()):
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        av = c.get("SQ_ACTIVE_INST_VALU", 0.0) or 1.0
        rows[p] = {
            "time_share": round(ns.get(p, 0.0) / tot_ns, 3),
            "parked_waitcnt_or_barrier": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 3),
            "issue_stalled": round(c.get("SQ_WAIT_INST_ANY", 0.0) / wc, 3),
            "issuing": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 3),
            "valu_active_per_wave_cycle": round(c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, 3),
            "valu_lane_fill": round(c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * av), 3),
            "lds_issue_stalled": round(c.get("SQ_WAIT_INST_LDS", 0.0) / wc, 3),
            "valu_insts": c.get("SQ_INSTS_VALU", 0.0),
        }
    res[cfg] = rows
json.dump(res, open(os.path.join(out, "stage_pmc.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
