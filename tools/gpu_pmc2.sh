#!/bin/bash
# memory-side counters (separate passes) for a kbench subset
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ONLY=${ONLY:-"conv7s1+relu@28->28,conv7s1@28->28"}
TAG=${TAG:-mem}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d gpurun_out/${TAG}_$i -o pmc -- \
        python tools/kbench.py --only "$ONLY" --rounds 1 --reps 2 > gpurun_out/${TAG}_$i.log 2>&1
    rc=$?; echo "== group $i ($grp) rc=$rc"; tail -2 gpurun_out/${TAG}_$i.log
    if [ $rc -ne 0 ]; then exit $rc; fi
done
