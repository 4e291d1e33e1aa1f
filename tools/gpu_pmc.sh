#!/bin/bash
# SQ / TCC counter passes over a kbench subset: one rocprofv3 --pmc pass per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ONLY=${ONLY:-"conv7s1+relu@28->28,conv7s1+relu(generic)@28->28"}
TAG=${TAG:-pmc}
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" ; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d gpurun_out/${TAG}_$i -o pmc -- \
        python tools/kbench.py --only "$ONLY" --rounds 1 --reps 2 > gpurun_out/${TAG}_$i.log 2>&1
    rc=$?; echo "== group $i rc=$rc"; tail -3 gpurun_out/${TAG}_$i.log
    if [ $rc -ne 0 ]; then exit $rc; fi
done
