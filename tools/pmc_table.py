"""Print per-kernel averages of every counter found in rocprofv3 --pmc output dirs.
    python tools/pmc_table.py gpurun_out/mem_*"""
import collections
import csv
import glob
import sys

res = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "Geo<" in k:
                k = k[k.index("Geo<"):k.index(">(") + 1]
            else:
                k = k.split("(")[0][-50:]
            res[(k, r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in res.items():
    print(key)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):.4g}")
