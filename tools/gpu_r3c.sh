#!/bin/bash
# round 3 session c: blocked Cholesky tests + pipeline tests, full-scale with the new solve,
# 2-rank gloo rehearsal of bench.py (rank-0 memory), solve_bench nb sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -k "solve or pipeline or world2 or var_chain" -x -v -s --timeout 200 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "peak|passed|failed" $O/pytest.log | tail -4
timeout -k 10 300 python tools/fullscale.py --n 60000 --m 10000 > $O/fullscale.json 2> $O/fullscale.err || { tail -20 $O/fullscale.err; exit 1; }
tail -c 1500 $O/fullscale.json
CGP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-f32 \
    --no-second --no-fullscale-f32 --fullscale-n 16384 --fullscale-m 4096 --cifar10-n 8192 > $O/bench_w2.json 2> $O/bench_w2.err || { tail -20 $O/bench_w2.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_w2.json').read().strip().splitlines()[-1])
print('w2 value', d['value'])
for k in ('fullscale','fullscale_cifar10'):
    f=d.get(k) or {}; print(k, {x: f.get(x) for x in f if x not in ('plan_kxx','plan_kxz')})
"
timeout -k 10 200 tools/bin/solve_bench 60000 2048 3072 4096 > $O/solve_bench.log 2>&1 || { tail -20 $O/solve_bench.log; exit 1; }
grep syrk $O/solve_bench.log
echo "== done"
