"""Summarise tools/pmc_ta.sh: per config, net_kernel's TA / TD busy cycles as a fraction of
the CU-cycles of its dispatches (GRBM_GUI_ACTIVE counts each XCD's clock;
TA_TA_BUSY_sum / TD_TD_BUSY_sum add one busy count per CU), and vector-memory read
wavefronts per pair.  Writes <out>/ta_pmc.json."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "*_ta"))):
    cfg = os.path.basename(d)[:-3]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    tot = {}
    for r in rows:
        if "net_kernel" not in r.get("Kernel_Name", ""):
            continue
        key = r["Counter_Name"]
        tot[key] = tot.get(key, 0.0) + float(r["Counter_Value"])
    if not tot:
        continue
    cus, xcds = 256, 8
    ns = 0.0
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "net_kernel" in r["Kernel_Name"]:
                ns += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    # GRBM_GUI_ACTIVE adds one count per XCD: its eighth over the dispatches' duration is
    # the clock (checked below), i.e. the CU-cycles each CU had
    gui = tot.get("GRBM_GUI_ACTIVE", 0.0) / xcds
    pairs = 3 * 1024 * 1024
    res[cfg] = {k: v for k, v in tot.items()}
    if gui:
        res[cfg]["ta_busy_frac_per_cu"] = tot.get("TA_TA_BUSY_sum", 0.0) / (gui * cus)
        res[cfg]["td_busy_frac_per_cu"] = tot.get("TD_TD_BUSY_sum", 0.0) / (gui * cus)
    res[cfg]["net_kernel_ns"] = ns
    res[cfg]["implied_clock_ghz"] = gui / ns if ns else None
    res[cfg]["flat_read_wavefronts_per_pair"] = tot.get("TA_FLAT_READ_WAVEFRONTS_sum", 0.0) / pairs
    res[cfg]["note"] = ("sums over the net_kernel dispatches of 3 B=1024 Kxz tiles; busy fractions "
                        "take GRBM_GUI_ACTIVE / 8 XCDs as each CU's cycles (implied_clock_ghz = that "
                        "over the dispatches' traced duration) and the TA/TD sums as one count per "
                        "CU (256)")
json.dump(res, open(os.path.join(out, "ta_pmc.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
