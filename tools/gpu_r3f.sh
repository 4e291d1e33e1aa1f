#!/bin/bash
# round 3 session f: GPU suite with the fp32 adaptive ReLU, fp32 A/B, bench kernel traces,
# then the driver's default bench command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2; do
  for data in rand mnist; do
    for v in noadapt default; do
      echo "== f32 $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --dtype f32 --data $data --configs mnist_paper_convnet_gp,mnist_paper_residual_cnn_gp,mnist_as_tf,cifar10 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace -o trace -- \
    python bench.py --steps 3 --no-cpu --no-fullscale --no-fullscale-cifar10 --no-second --no-f32 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace_tf -o trace -- \
    python bench.py --config mnist_as_tf --steps 3 --no-cpu --no-fullscale --no-fullscale-cifar10 --no-f32 > $O/trace_tf.log 2>&1 || { tail -20 $O/trace_tf.log; exit 1; }
tail -1 $O/trace.log | cut -c1-300
T0=$SECONDS; timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; echo "bench wall $((SECONDS - T0)) s"
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('value', d['value'], 'tf', d['mnist_as_tf']['value'], 'roof', r['frac'], r['avg_ms'], r['valu_issue_frac'], r['valu_insts_per_pair'])
for k in ('fullscale','fullscale_f32','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in ('kxx_s','kxz_s','solve_s','total_s','spot_check_hip_vs_hip_max_rel_err','spot_vs_f64_max_rel_err')})
print('f32', d['f32']); print('solve', d.get('solve'))
"
echo "== done"
