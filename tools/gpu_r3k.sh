#!/bin/bash
# round 3 session k: A/B of the one-chain adaptive ReLU (CGP_RELU_CHAIN), the undefined
# conv results (CGP_NET_RES_UNDEF), opaque LDS bases (CGP_NET_LDS_BASE), all three, and
# the per-pair-segment adaptive ReLU in multi-pair stages (CGP_RELU_ADAPT_MP); parity of the
# new builds, then VALU instruction counts (PMC) of base vs all3, and an I-cache pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
V=${VARS:-"base chain undef ldsb all3 mp"}
for v in ${PARITY:-chain all3}; do
  echo "== parity $v"
  CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x -k "netfuse or e2e or first_stage or zero or compiled" --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1
  rc=$?; tail -1 $O/parity_$v.log
  if [ $rc -gt 1 ]; then tail -20 $O/parity_$v.log; exit $rc; fi
done
for rep in 1 2; do
  for v in $V; do
    echo "== $v rep=$rep"
    CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --reps 3 2>&1 | grep -v amdgpu.ids | cut -c1-70 || exit $?
  done
done
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"
for v in ${PMC:-base all3}; do
  for cfg in mnist_paper_convnet_gp mnist_as_tf; do
    CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE -f csv -d $O/pmc_${v}_$cfg -o pmc -- python3 tools/netbench.py --configs $cfg --reps 1 > $O/pmc_${v}_$cfg.log 2>&1
    rc=$?; echo "== pmc $v $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_${v}_$cfg.log; exit $rc; }
  done
done
for v in base chain; do
  CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES -f csv -d $O/ic_$v -o pmc -- python3 tools/netbench.py --configs mnist_as_tf --reps 1 > $O/ic_$v.log 2>&1
  rc=$?; echo "== icache $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/ic_$v.log; exit 0; }
done
echo "== done"
