#!/bin/bash
# L2 behaviour of the whole-network kernel: TCC hit/miss and memory-side read requests
# (separate rocprofv3 passes) over tools/netbench.py on one config
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-mnist_paper_convnet_gp}
TAG=${TAG:-l2}
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d gpurun_out/${TAG}_$i -o pmc -- \
        python tools/netbench.py --configs $CFG --reps 1 > gpurun_out/${TAG}_$i.log 2>&1
    rc=$?; echo "== group $i ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_$i.log; exit $rc; fi
done
python3 - "$TAG" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
tot = {}
n = {}
for f in glob.glob(f"gpurun_out/{tag}_*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "net_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            n[r["Counter_Name"]] = n.get(r["Counter_Name"], 0) + 1
for k in sorted(tot):
    print(f"{k:34s} {tot[k]:.4e}  (dispatches {n[k]})")
h, m = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
if h + m:
    print(f"L2 hit rate {h / (h + m):.3f}")
PY
