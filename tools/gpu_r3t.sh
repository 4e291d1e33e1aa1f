#!/bin/bash
# round 3 session t: wave priority around the conv's memory phase (CGP_NET_PRIO=1 / 3) vs
# the shipped kernel; tools/netbench.py, one B = 1024 Kxz tile per config, fp64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base prio1 prio3; do
    echo "== $v rep=$rep"
    CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --reps 3 2>&1 | grep -v amdgpu.ids | cut -c1-70 || exit $?
  done
done
echo "== done"
