#!/bin/bash
# round 3 session o: the bound-build tests (memory budget included), then a 4-rank gloo
# rehearsal of bench.py on the one GPU with the bound Gram builds (weak-scaling leg and the
# full-scale pipeline at reduced sizes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q -k "bound_build or world2" --timeout 200 --timeout-method thread > $O/pytest_bound.log 2>&1 || { tail -30 $O/pytest_bound.log; exit 1; }
tail -1 $O/pytest_bound.log
CGP_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu --no-f32 \
    --no-second --no-fullscale-f32 --fullscale-n 24576 --fullscale-m 8192 --cifar10-n 12288 > $O/bench_w4.json 2> $O/bench_w4.err || { tail -20 $O/bench_w4.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_w4.json').read().strip().splitlines()[-1])
print('w4 value', d['value'], d['config'])
for k in ('fullscale','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in f if x not in ('note','data')})
"
echo "== done"
