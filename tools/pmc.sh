#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, each under its own timeout):
#   net_kernel on one B=1024 Kxz tile per config (tools/netbench.py --reps 1: 3 tile
#   evaluations) and the standalone Conv2d stencil (tools/stencil_once.py: 3 launches).
# Summarised by tools/pmc_r2.py into net_pmc.json (profiles/r<round>/).
#   PMC_CFGS="mnist_paper_convnet_gp mnist_as_tf cifar10" OUT=gpurun_out/x bash tools/pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_r2}
CFGS=${PMC_CFGS:-"mnist_paper_convnet_gp mnist_as_tf cifar10"}
mkdir -p $OUT
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
run() {   # tag counters cmd...
    local tag=$1 ctr=$2; shift 2
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -f csv -d $OUT/$tag -o pmc -- "$@" > $OUT/$tag.log 2>&1
    local rc=$?
    echo "== $tag ($ctr) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
}
for cfg in $CFGS; do
    run ${cfg}_fetch "FETCH_SIZE" python3 tools/netbench.py --configs $cfg --reps 1
    run ${cfg}_write "WRITE_SIZE" python3 tools/netbench.py --configs $cfg --reps 1
    run ${cfg}_sq "$SQ GRBM_GUI_ACTIVE" python3 tools/netbench.py --configs $cfg --reps 1
done
run stencil_fetch "FETCH_SIZE" python3 tools/stencil_once.py
run stencil_write "WRITE_SIZE" python3 tools/stencil_once.py
