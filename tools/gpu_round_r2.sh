#!/bin/bash
# One round-end measurement session on the GPU box (each step under its own timeout,
# stopping at the first failure):  parity tests -> PMC passes (tools/gpu_pmc_r2.sh, summary
# written to profiles/r2/net_pmc.json on the box and copied to gpurun_out/) -> bench.py
# (reads that summary) -> rocprofv3 kernel trace of the bench command.
#   TAG=r2h bash tools/gpu_round_r2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
OUT=$O/pmc bash tools/gpu_pmc_r2.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pmc_r2.py $O/pmc profiles/r2/net_pmc.json > /dev/null && cp profiles/r2/net_pmc.json $O/net_pmc.json || exit 1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
# one trace per config, so each stats CSV's net_kernel row is that config's alone and
# compares with the bench line's roofline.avg_ms for it
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace -o trace -- \
    python bench.py --steps 3 --no-cpu --no-fullscale --no-second --no-f32 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/trace_tf -o trace -- \
    python bench.py --config mnist_as_tf --steps 3 --no-cpu --no-fullscale --no-f32 > $O/trace_tf.log 2>&1 || { tail -20 $O/trace_tf.log; exit 1; }
echo "== done"
