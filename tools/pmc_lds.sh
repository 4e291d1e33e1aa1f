#!/bin/bash
# Where net_kernel's waves spend their cycles, and its LDS bank conflicts: one rocprofv3
# --pmc pass per config (8 SQ counters + GRBM) over one B=1024 Kxz tile x 3
# (tools/netbench.py --reps 1).  Summary: tools/pmc_lds.py -> lds_pmc.json.
#   OUT=gpurun_out/x PMC_CFGS="mnist_paper_convnet_gp" bash tools/pmc_lds.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_lds}
CFGS=${PMC_CFGS:-"mnist_paper_convnet_gp mnist_as_tf cifar10"}
mkdir -p $OUT
for cfg in $CFGS; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -f csv -d $OUT/${cfg}_lds \
        -o pmc -- python3 tools/netbench.py --configs $cfg --reps 1 > $OUT/${cfg}_lds.log 2>&1
    rc=$?
    echo "== ${cfg}_lds rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/${cfg}_lds.log; exit $rc; fi
done
python3 tools/pmc_lds.py $OUT
