#!/bin/bash
# round 3 session e: GPU suite on the adaptive-ReLU default, A/B against CGP_RELU_ADAPT=0,
# refreshed PMC passes (profiles/r3/net_pmc.json), then the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_adaptmp.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multi.py tests/test_gpu_fullgeom.py -q -x -k "netfuse or e2e or bench_geometry or world2 or full_scale" --timeout 200 --timeout-method thread > $O/ab_pytest_adaptmp.log 2>&1 || { echo "pytest adaptmp failed"; tail -20 $O/ab_pytest_adaptmp.log; exit 1; }
echo "adaptmp: $(tail -1 $O/ab_pytest_adaptmp.log)"
for rep in 1 2; do
  for data in rand mnist; do
    for v in noadapt default adaptmp; do
      echo "== $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --data $data --configs mnist_paper_convnet_gp,mnist_paper_residual_cnn_gp,mnist_as_tf,cifar10 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
OUT=$O/pmc bash tools/gpu_pmc_r2.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
mkdir -p profiles/r3 && python3 tools/pmc_r2.py $O/pmc profiles/r3/net_pmc.json > /dev/null && cp profiles/r3/net_pmc.json $O/net_pmc.json || exit 1
T0=$SECONDS; timeout -k 10 900 python bench.py --no-fullscale-f32 --no-fullscale-cifar10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; echo "bench wall $((SECONDS - T0)) s"
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('value', d['value'], 'tf', d['mnist_as_tf']['value'], 'roof', r['frac'], r['avg_ms'], r['valu_issue_frac'], r['valu_insts_per_pair'], r['traffic'])
f=d['fullscale']; print('fullscale', {x: f.get(x) for x in ('kxx_s','kxz_s','solve_s','total_s','spot_check_hip_vs_hip_max_rel_err')})
print('f32', d['f32'])
"
echo "== done"
