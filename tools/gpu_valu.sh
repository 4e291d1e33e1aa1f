#!/bin/bash
# VALU busy / lane utilisation / LDS and VMEM latency of the whole-network kernel (one
# rocprofv3 --pmc pass per counter group; rocprofv3 does not split groups itself).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-valu}
CFGS=${CFGS:-mnist_paper_convnet_gp}
i=0
for grp in "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d gpurun_out/${TAG}_$i -o pmc -- \
        python tools/netbench.py --configs $CFGS --reps 1 > gpurun_out/${TAG}_$i.log 2>&1
    rc=$?; echo "== group $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 gpurun_out/${TAG}_$i.log; exit $rc; fi
done
