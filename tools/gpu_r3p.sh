#!/bin/bash
# round 3 session p: A/B of the fine-grained adaptive ReLU (CGP_RELU_FINE: degrees 6-13 by
# a binary search of wave votes) against the shipped 7/9/11/13 form (mp), with and without
# the multi-pair per-segment vote; parity of the new build; VALU counts (PMC)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
for v in fine finenomp; do
  echo "== parity $v"
  CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -q -x -k "netfuse or e2e or first_stage or zero or compiled or bound or bench_geometry" --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1
  rc=$?; tail -1 $O/parity_$v.log
  if [ $rc -ne 0 ]; then tail -20 $O/parity_$v.log; exit $rc; fi
done
for rep in 1 2; do
  for data in rand mnist; do
    for v in mp fine finenomp; do
      echo "== $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --reps 3 --data $data 2>&1 | grep -v amdgpu.ids | cut -c1-70 || exit $?
    done
  done
done
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"
for v in mp fine; do
  for cfg in mnist_paper_convnet_gp mnist_as_tf; do
    CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ GRBM_GUI_ACTIVE -f csv -d $O/pmc_${v}_$cfg -o pmc -- python3 tools/netbench.py --configs $cfg --reps 1 > $O/pmc_${v}_$cfg.log 2>&1
    rc=$?; echo "== pmc $v $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_${v}_$cfg.log; exit $rc; }
  done
done
echo "== done"
