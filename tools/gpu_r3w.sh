#!/bin/bash
# round 3 session w: the wave-priority default (CGP_NET_PRIO=2): GPU suite, smoke, refreshed
# PMC passes (profiles/r3/net_pmc.json), bench kernel traces, the driver's default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
OUT=$O/pmc bash tools/gpu_pmc_r2.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
mkdir -p profiles/r3 && python3 tools/pmc_r2.py $O/pmc profiles/r3/net_pmc.json > /dev/null && cp profiles/r3/net_pmc.json $O/net_pmc.json || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace -o trace -- \
    python bench.py --steps 3 --no-cpu --no-fullscale --no-fullscale-cifar10 --no-second --no-f32 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace_tf -o trace -- \
    python bench.py --config mnist_as_tf --steps 3 --no-cpu --no-fullscale --no-fullscale-cifar10 --no-f32 > $O/trace_tf.log 2>&1 || { tail -20 $O/trace_tf.log; exit 1; }
T0=$SECONDS; timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; echo "bench wall $((SECONDS - T0)) s"
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; m=d['mnist_as_tf']; print('value', d['value'], 'step', d['ms_per_step'], 'net', r['avg_ms'], 'frac', r['frac'], 'issue', r.get('valu_issue_frac'), '| tf', m['value'], 'step', m['ms_per_step'], 'frac', m['roofline']['frac'])
for k in ('fullscale','fullscale_f32','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in ('kxx_s','kxz_s','solve_s','total_s','spot_check_hip_vs_hip_max_rel_err')})
print('f32', {k: v['value'] for k, v in d['f32'].items() if isinstance(v, dict)})
"
echo "== done"
