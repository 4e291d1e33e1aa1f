#!/bin/bash
# round 3 sessions x/y: wave-priority span — variance loads and window reads (default) vs the
# variance loads only (x: CGP_NET_PRIO_SPAN=1) or the window reads only (y: =2), each also on cifar10, vs off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in ${VARS:-noprio def span2 span2all}; do
    echo "== $v rep=$rep"
    CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --reps 3 2>&1 | grep -v amdgpu.ids | cut -c1-70 || exit $?
  done
done
echo "== done"
