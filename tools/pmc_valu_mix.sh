#!/bin/bash
# VALU instruction mix of net_kernel per stage and library variant (verdict r5 item 2):
# one rocprofv3 --pmc pass per (variant, config) with SQ_INSTS_VALU and its fp64 / integer
# class counters over one B=1024 Kxz tile x 3 (tools/netbench.py --reps 1); summary by
# tools/pmc_valu_mix.py -> <OUT>/valu_mix.json.  Variants: "cur" = lib/libcnngp.so, NAME =
# cnn-gp_amd/lib/ab/lib_NAME.so.
#   VARIANTS="base cur" PMC_CFGS="mnist_as_tf" OUT=gpurun_out/x bash tools/pmc_valu_mix.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/valu_mix}
CFGS=${PMC_CFGS:-"mnist_paper_convnet_gp mnist_as_tf cifar10"}
VARIANTS=${VARIANTS:-cur}
CTR=${VALU_CTR:-"SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"}
mkdir -p $OUT
for v in $VARIANTS; do
    if [ "$v" = cur ]; then export CNNGP_LIB=$PWD/cnn-gp_amd/lib/libcnngp.so
    else export CNNGP_LIB=$PWD/cnn-gp_amd/lib/ab/lib_$v.so; fi
    for cfg in $CFGS; do
        tag=${v}_${cfg}
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR -f csv -d $OUT/$tag -o pmc -- \
            python3 tools/netbench.py --configs $cfg --reps 1 ${NB_EXTRA:-} > $OUT/$tag.log 2>&1
        rc=$?
        echo "== $tag rc=$rc"
        if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
    done
done
python3 tools/pmc_valu_mix.py $OUT
