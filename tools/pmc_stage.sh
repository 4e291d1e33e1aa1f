#!/bin/bash
# Where each net_kernel stage program's waves spend their cycles (verdict r5 item 5: the
# cifar10 head): one rocprofv3 --pmc pass per config over one B=1024 Kxz tile x 3
# (tools/netbench.py --reps 1) with the wave-cycle counters, split per program by
# tools/pmc_stage.py -> <OUT>/stage_pmc.json.
#   PMC_CFGS="cifar10 mnist_as_tf" OUT=gpurun_out/x bash tools/pmc_stage.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_stage}
CFGS=${PMC_CFGS:-"cifar10 mnist_as_tf"}
mkdir -p $OUT
for cfg in $CFGS; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU \
        SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -f csv -d $OUT/${cfg}_st -o pmc -- \
        python3 tools/netbench.py --configs $cfg --reps 1 > $OUT/${cfg}_st.log 2>&1
    rc=$?
    echo "== ${cfg}_st rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/${cfg}_st.log; exit $rc; fi
done
python3 tools/pmc_stage.py $OUT
