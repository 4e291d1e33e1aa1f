#!/bin/bash
# round 3 session d: the driver's default bench command, then one rocprofv3 kernel trace per
# config of the bench's Kxx legs (profiles/r3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
T0=$SECONDS; timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; echo "bench wall $((SECONDS - T0)) s"

python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'tf', d['mnist_as_tf']['value'], 'roof', d['roofline']['frac'], d['roofline']['avg_ms'])
for k in ('fullscale','fullscale_f32','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in f if x not in ('plan_kxx','plan_kxz','note','data')})
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['mnist_as_tf']['cpu_baseline']['value'])
"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace -o trace -- \
    python bench.py --steps 3 --no-cpu --no-fullscale --no-fullscale-cifar10 --no-second --no-f32 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace_tf -o trace -- \
    python bench.py --config mnist_as_tf --steps 3 --no-cpu --no-fullscale --no-fullscale-cifar10 --no-f32 > $O/trace_tf.log 2>&1 || { tail -20 $O/trace_tf.log; exit 1; }
echo "== done"
# A/B: range-adaptive ReLU polynomial (CGP_RELU_ADAPT=1) against the same source without it
for v in base adapt; do
  CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -q -x -k "netfuse or e2e or bench_geometry" --timeout 200 --timeout-method thread > $O/ab_pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -20 $O/ab_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/ab_pytest_$v.log)"
done
for rep in 1 2; do
  for data in rand mnist; do
    for v in base adapt; do
      echo "== $v data=$data rep=$rep"
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so timeout -k 10 200 python tools/netbench.py --data $data --configs mnist_paper_convnet_gp,mnist_as_tf,cifar10 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
echo "== ab done"
