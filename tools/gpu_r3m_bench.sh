#!/bin/bash
# round 3 session m: the driver's default bench command on the final code
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
T0=$SECONDS; timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; echo "bench wall $((SECONDS - T0)) s"
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('value', d['value'], 'tf', d['mnist_as_tf']['value'], 'roof', r['frac'], r['avg_ms'], r['valu_issue_frac'], r['valu_insts_per_pair'])
for k in ('fullscale','fullscale_f32','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in ('kxx_s','kxz_s','solve_s','total_s','spot_check_hip_vs_hip_max_rel_err','spot_vs_f64_max_rel_err')})
print('f32', d['f32']); print('solve', d.get('solve'))
"
echo "== done"
