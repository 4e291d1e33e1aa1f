#!/bin/bash
# round 3 session h: A/B of the whole-chain Horner asm blocks (CGP_HORNER_ASM=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_hasm.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multi.py -q -x -k "netfuse or e2e or bench_geometry or world2" --timeout 200 --timeout-method thread > $O/ab_pytest_hasm.log 2>&1 || { echo "pytest hasm failed"; tail -20 $O/ab_pytest_hasm.log; exit 1; }
echo "hasm: $(tail -1 $O/ab_pytest_hasm.log)"
for rep in 1 2 3; do
  for v in default hasm; do
    echo "== $v rep=$rep"
    CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --configs mnist_paper_convnet_gp,mnist_paper_residual_cnn_gp,mnist_as_tf,cifar10 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
echo "== done"
