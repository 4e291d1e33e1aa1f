#!/bin/bash
# round 3, first GPU session: new geometry tests + full gpu suite + smoke + bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullgeom.py -x -v -s --timeout 200 --timeout-method thread \
    > $O/pytest_fullgeom.log 2>&1 || { tail -30 $O/pytest_fullgeom.log; exit 1; }
grep -E "worst|passed|failed" $O/pytest_fullgeom.log | tail -8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'tf', d['mnist_as_tf']['value'])
for k in ('fullscale','fullscale_f32','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in ('kxx_s','kxz_s','solve_s','total_s','fullscale_wall_s')})
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['cpu_baseline']['host_cpus'])
"
echo "== done"
