#!/bin/bash
# round 3 session g: posterior variance through the strip pipeline (gather_kxz), and a
# 4-rank gloo rehearsal of bench.py on the one GPU (rank-0 memory, Kxz shares)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python tools/fullscale.py --n 20000 --m 5000 --pred-var > $O/fullscale_predvar.json 2> $O/fullscale_predvar.err || { tail -20 $O/fullscale_predvar.err; exit 1; }
tail -c 1200 $O/fullscale_predvar.json
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
