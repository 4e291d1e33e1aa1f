#!/bin/bash
# Executed fp64 arithmetic of net_kernel: one rocprofv3 --pmc pass per config with the
# gfx950 VALU flop counters (SQ_INSTS_VALU_FLOPS_FP64 / _FP64_TRANS count flops per lane
# executed; the FMA / ADD / MUL / TRANS wave-instruction counts beside them), over one
# B=1024 Kxz tile x 3 (tools/netbench.py --reps 1).  Summary: tools/pmc_flops.py ->
# flops_pmc.json.
#   OUT=gpurun_out/x bash tools/pmc_flops.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_flops}
CFGS=${PMC_CFGS:-"mnist_paper_convnet_gp mnist_as_tf cifar10"}
mkdir -p $OUT
for cfg in $CFGS; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP64 \
        SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 \
        SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -f csv -d $OUT/${cfg}_fl -o pmc -- \
        python3 tools/netbench.py --configs $cfg --reps 1 > $OUT/${cfg}_fl.log 2>&1
    rc=$?
    echo "== ${cfg}_fl rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/${cfg}_fl.log; exit $rc; fi
done
python3 tools/pmc_flops.py $OUT
