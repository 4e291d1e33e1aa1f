#!/bin/bash
# round 3 session m: GPU suite + smoke on the multi-pair adaptive ReLU default
# (CGP_RELU_ADAPT_MP=1), refreshed PMC passes (profiles/r3/net_pmc.json) and the bench's
# kernel traces; the bench itself runs in tools/gpu_r3m_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3m
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
tail -1 $O/trace.log | cut -c1-300
echo "== done"
