#!/bin/bash
# round 3 session d: the driver's default bench command, then one rocprofv3 kernel trace per
# config of the bench's Kxx legs (profiles/r3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
/usr/bin/time -f "bench wall %e s" timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.err
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
