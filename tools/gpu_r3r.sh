#!/bin/bash
# round 3 session r: register target of the multi-pair stage programs (CGP_NET_PROG_WPE_MP=4:
# no spills, fewer waves) against the shipped 5 (spills with the per-segment vote) and the
# per-segment vote off; the two ResNets, per-stage times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
echo "== parity mpw4"
CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_mpw4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x -k "netfuse or e2e or first_stage or compiled" --timeout 120 --timeout-method thread > $O/parity_mpw4.log 2>&1
rc=$?; tail -1 $O/parity_mpw4.log; [ $rc -ne 0 ] && { tail -20 $O/parity_mpw4.log; exit $rc; }
for rep in 1 2; do
  for data in rand mnist; do
    for v in base mpw4 nomp; do
      echo "== $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --reps 3 --data $data --per-stage --configs mnist_as_tf,cifar10 2>&1 | grep -v amdgpu.ids | cut -c1-90 || exit $?
    done
  done
done
echo "== done"
