#!/bin/bash
# A/B timing of libcnngp builds under cnn-gp_amd/lib/ab/lib_<name>.so (CNNGP_LIB), each
# checked by the whole-network parity tests first.   VARIANTS="a b" bash tools/variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-$(ls cnn-gp_amd/lib/ab | sed -n 's/^lib_\(.*\)\.so$/\1/p')}; do
  echo "== $v"
  export CNNGP_LIB=$PWD/cnn-gp_amd/lib/ab/lib_$v.so
  # builds before the quartered-map ReLU (relu_q_n) read plain variance maps
  case " ${PLAIN_MAPS:-} " in *" $v "*) export CGP_NET_QUARTER=0 ;; *) export CGP_NET_QUARTER=1 ;; esac
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "netfuse or e2e" --timeout 120 --timeout-method thread 2>&1 | tail -1
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  timeout -k 10 200 python tools/netbench.py ${NB_ARGS:-} 2>&1 | grep -v amdgpu.ids || exit $?
done
