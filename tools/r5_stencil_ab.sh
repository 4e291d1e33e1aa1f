#!/bin/bash
# A/B of the stencil kernel's LDS-staged 16-byte output stores (CGP_GEO_STAGE_OUT=1,
# lib/ab/lib_stgout.so) against the shipped library: the variant's per-op conv parity
# tests first, then tools/stencil_once.py (bench.py's conv_stencil_roofline launch) per
# library, three rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_stencil}
mkdir -p "$O"
timeout -k 10 300 env CNNGP_LIB=$PWD/cnn-gp_amd/lib/ab/lib_stgout.so python -u -m pytest \
    tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "conv or layer" \
    > "$O/stgout_tests.log" 2>&1 || { echo "stgout tests rc=$?"; tail -n 20 "$O/stgout_tests.log"; exit 1; }
tail -n 1 "$O/stgout_tests.log"
for rep in 1 2 3; do for v in cur stgout; do
    lib=$PWD/cnn-gp_amd/lib/libcnngp.so; [ $v = stgout ] && lib=$PWD/cnn-gp_amd/lib/ab/lib_stgout.so
    timeout -k 10 120 env CNNGP_LIB=$lib python tools/stencil_once.py > "$O/st_${v}_$rep.log" 2>&1 || exit 1
    echo "-- $v $rep: $(grep -v amdgpu.ids "$O/st_${v}_$rep.log" | tail -n 1)"
done; done
