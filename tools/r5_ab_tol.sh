set -u
O=gpurun_out/r5d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 env CNNGP_LIB=$PWD/cnn-gp_amd/lib/ab/lib_tol.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_fullgeom.py -q --timeout 200 --timeout-method thread -k "netfuse or e2e or program or scale or full" > $O/tol_tests.log 2>&1
rc=$?; echo "tol tests rc=$rc"; tail -n 30 $O/tol_tests.log | grep -E "passed|failed|Error|assert" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for data in rand mnist; do for rep in 1 2; do for v in cur tol; do
  lib=$PWD/cnn-gp_amd/lib/libcnngp.so; [ $v = tol ] && lib=$PWD/cnn-gp_amd/lib/ab/lib_tol.so
  timeout -k 10 200 env CNNGP_LIB=$lib python tools/netbench.py --configs mnist_paper_convnet_gp,mnist_as_tf,cifar10 --data $data > $O/ab_${v}_${data}_$rep.log 2>&1 || exit 1
  echo "-- $v $data $rep"; grep -v amdgpu.ids $O/ab_${v}_${data}_$rep.log | tail -n 4
done; done; done
