#!/bin/bash
# A/B of one library variant (cnn-gp_amd/lib/ab/lib_$V.so, tools/build_variant.sh) against
# the shipped library: the variant's whole-network parity tests first, then
# tools/netbench.py (one B = 1024 Kxz tile per config) on uniform and MNIST-like images,
# two rounds, alternating.
#   V=tol2 O=gpurun_out/x bash tools/ab_variant.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${V:?variant name}
O=${O:-gpurun_out/ab_$V}
CFGS=${CFGS:-mnist_paper_convnet_gp,mnist_as_tf,cifar10}
mkdir -p "$O"
VL=$PWD/cnn-gp_amd/lib/ab/lib_$V.so
if [ -z "${SKIP_TESTS:-}" ]; then      # SKIP_TESTS=1: timing probes with wrong results
    timeout -k 10 300 env CNNGP_LIB=$VL python -u -m pytest tests/test_gpu_parity.py \
        tests/test_gpu_scale.py tests/test_gpu_fullgeom.py -q --timeout 200 \
        --timeout-method thread -k "netfuse or e2e or program or scale or full" \
        > "$O/${V}_tests.log" 2>&1
    rc=$?
    echo "$V tests rc=$rc: $(tail -n 1 "$O/${V}_tests.log")"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for data in rand mnist; do for rep in 1 2; do for v in cur $V; do
    lib=$PWD/cnn-gp_amd/lib/libcnngp.so; [ $v = $V ] && lib=$VL
    timeout -k 10 200 env CNNGP_LIB=$lib python tools/netbench.py --configs $CFGS --data $data \
        ${NB_ARGS:-} > "$O/ab_${v}_${data}_$rep.log" 2>&1 || exit 1
    echo "-- $v $data $rep"; grep -v amdgpu.ids "$O/ab_${v}_${data}_$rep.log" | tail -n 3 | cut -c1-70
done; done; done
