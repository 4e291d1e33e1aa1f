#!/bin/bash
# round 3 session u: wave priority refinements: CGP_NET_PRIO=3 everywhere / head stage only
# (CGP_NET_PRIO_MP=0) / =2, vs the shipped kernel; parity of prio3; netbench --per-stage,
# uniform and MNIST-like images
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_prio3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x -k "netfuse or e2e or first_stage or compiled or bound" --timeout 120 --timeout-method thread > $O/parity_prio3.log 2>&1
rc=$?; tail -1 $O/parity_prio3.log; [ $rc -ne 0 ] && { tail -20 $O/parity_prio3.log; exit $rc; }
for rep in 1 2; do
  for data in rand mnist; do
    for v in base prio3 prio3h prio2; do
      echo "== $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --reps 3 --data $data --per-stage 2>&1 | grep -v amdgpu.ids | cut -c1-70 || exit $?
    done
  done
done
echo "== done"
