#!/bin/bash
# round 3 session i: GPU suite, smoke and the driver's default bench command on the final code
# (float32 full-scale leg widens Kxx in place)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
T0=$SECONDS; timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; echo "bench wall $((SECONDS - T0)) s"
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('value', d['value'], 'tf', d['mnist_as_tf']['value'], 'roof', r['frac'], r['avg_ms'])
for k in ('fullscale','fullscale_f32','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in ('kxx_s','kxz_s','solve_s','total_s','rank0_peak_gather_solve_over_kxx','spot_check_hip_vs_hip_max_rel_err','spot_vs_f64_max_rel_err')})
"
echo "== done"
