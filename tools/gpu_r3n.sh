#!/bin/bash
# round 3 session n: Gram builds from one build's variance maps (ModelKern.bind): the new
# bit-equality tests, the GPU suite, then bench.py (default command) on the new step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "bound_build" --timeout 200 --timeout-method thread > $O/pytest_bound.log 2>&1 || { tail -30 $O/pytest_bound.log; exit 1; }
tail -1 $O/pytest_bound.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
T0=$SECONDS; timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; echo "bench wall $((SECONDS - T0)) s"
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; m=d['mnist_as_tf']; print('value', d['value'], 'step', d['ms_per_step'], 'net', r['avg_ms'], 'x', r['launches'], '| tf', m['value'], 'step', m['ms_per_step'], 'net', m['roofline']['avg_ms'])
for k in ('fullscale','fullscale_f32','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in ('kxx_s','kxz_s','solve_s','total_s','rank0_peak_gb_kxx_build','rank0_peak_gb_gather_solve','rank0_peak_gb_kxz','spot_check_hip_vs_hip_max_rel_err')})
print('f32', {k: v['value'] for k, v in d['f32'].items() if isinstance(v, dict)})
"
echo "== done"
