#!/bin/bash
# round 3 session j: factored variance maps (CGP_RELU_FACT) — GPU suite on the default
# (factored) library, then netbench A/B against the unfactored build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for data in rand mnist; do
    for v in nofact fact noslow; do
      [ $v = noslow ] && [ $data = mnist ] && continue
      echo "== $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --data $data --configs mnist_paper_convnet_gp,mnist_paper_residual_cnn_gp,mnist_as_tf,cifar10 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
echo "== ab done"
