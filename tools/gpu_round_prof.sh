#!/bin/bash
# Round profile session: bench JSON lines, rocprofv3 kernel stats of the bench command,
# FETCH/WRITE PMC passes of the fused kernel per config (traffic per launch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r1}
CFGS=${CFGS:-mnist_paper_convnet_gp mnist_as_tf}
for c in $CFGS; do
    extra=""; [ "$c" = "cifar10" ] && extra="--n 2048 --no-solve"
    timeout -k 10 300 python bench.py --config $c $extra > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || exit $?
    tail -1 gpurun_out/${TAG}_bench_$c.json
done
c0=$(echo $CFGS | cut -d' ' -f1)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${TAG}_trace -o trace -- \
    python bench.py --config $c0 --steps 2 --no-cpu > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
echo "== trace ok"
for c in $CFGS; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -f csv -d gpurun_out/${TAG}_${ctr}_$c -o pmc -- \
            python tools/netbench.py --configs $c --reps 1 > gpurun_out/${TAG}_${ctr}_$c.log 2>&1 || exit $?
    done
    python tools/pmc_traffic.py $c 1024 torch.float64 gpurun_out/${TAG}_FETCH_SIZE_$c gpurun_out/${TAG}_WRITE_SIZE_$c gpurun_out/${TAG}_net_traffic.json || exit $?
done
