#!/bin/bash
# Whole-network kernel: timing, rocprofv3 kernel stats, SQ counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-net}
CFGS=${CFGS:-mnist_paper_convnet_gp,mnist_as_tf}
NB_ARGS=${NB_ARGS:-}
timeout -k 10 300 python tools/netbench.py --configs $CFGS $NB_ARGS > gpurun_out/${TAG}_time.log 2>&1 || exit $?
cat gpurun_out/${TAG}_time.log
if [[ ${STEPS:-trace,pmc} == *trace* ]]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${TAG}_trace -o trace -- \
        python tools/netbench.py --configs $CFGS --reps 2 $NB_ARGS > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
    echo "== trace ok"
fi
if [[ ${STEPS:-trace,pmc} == *pmc* ]]; then
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT" \
           "TCC_HIT_sum TCC_MISS_sum" ; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d gpurun_out/${TAG}_pmc_$i -o pmc -- \
        python tools/netbench.py --configs $CFGS --reps 1 $NB_ARGS > gpurun_out/${TAG}_pmc_$i.log 2>&1
    rc=$?; echo "== group $i rc=$rc"; tail -2 gpurun_out/${TAG}_pmc_$i.log
    if [ $rc -ne 0 ]; then exit $rc; fi
done
fi
