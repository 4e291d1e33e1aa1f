"""Summarise tools/pmc_lds.sh: per config, net_kernel's wave-cycle split (parked on
s_waitcnt / barrier, issue-stalled, issuing), the LDS share of the stalls, and LDS bank
conflicts as extra cycles over all LDS-array cycles.  Writes <out>/lds_pmc.json."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "*_lds"))):
    cfg = os.path.basename(d)[:-4]
    tot = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "net_kernel" in r.get("Kernel_Name", ""):
                k = r["Counter_Name"]
                tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
    if not tot:
        continue
    wc = tot.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    idx = tot.get("SQ_LDS_IDX_ACTIVE", 0.0) or 1.0
    res[cfg] = dict(tot)
    res[cfg].update(
        wait_any_frac=tot.get("SQ_WAIT_ANY", 0.0) / wc,
        wait_inst_any_frac=tot.get("SQ_WAIT_INST_ANY", 0.0) / wc,
        active_inst_any_frac=tot.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
        wait_inst_lds_frac=tot.get("SQ_WAIT_INST_LDS", 0.0) / wc,
        active_inst_lds_frac=tot.get("SQ_ACTIVE_INST_LDS", 0.0) / wc,
        lds_bank_conflict_frac=tot.get("SQ_LDS_BANK_CONFLICT", 0.0) / idx,
        note="fractions of SQ_WAVE_CYCLES over the net_kernel dispatches of 3 B=1024 Kxz "
             "tiles; lds_bank_conflict_frac = extra conflict cycles / all LDS-array cycles")
json.dump(res, open(os.path.join(out, "lds_pmc.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
