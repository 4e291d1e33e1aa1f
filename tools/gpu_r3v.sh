#!/bin/bash
# round 3 session v: wave priority as the default (CGP_NET_PRIO=2 on maps up to 28x28) vs
# off, vs also around the elementwise ops' loads (CGP_NET_PRIO_ELEM=1), vs on every map size
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_pe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x -k "netfuse or e2e or first_stage or compiled" --timeout 120 --timeout-method thread > $O/parity_pe.log 2>&1
rc=$?; tail -1 $O/parity_pe.log; [ $rc -ne 0 ] && { tail -20 $O/parity_pe.log; exit $rc; }
for rep in 1 2; do
  for data in rand mnist; do
    for v in noprio def pe allhw; do
      echo "== $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --reps 3 --data $data 2>&1 | grep -v amdgpu.ids | cut -c1-70 || exit $?
    done
  done
done
echo "== done"
