#!/bin/bash
# round 3 session l: bench.py Kxx 4096² at tile 1024 / 2048 / 4096 (one launch per tile:
# fewer launch tails and inter-tile gaps), default library and the multi-pair adaptive
# ReLU build (CGP_RELU_ADAPT_MP=1), twice each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
for rep in 1 2; do
  for lib in base mp; do
    for t in 1024 2048 4096; do
      CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$lib.so timeout -k 10 300 python bench.py --tile $t --no-fullscale --no-cpu --no-f32 --no-solve > $O/b_${lib}_${t}_$rep.json 2> $O/b_${lib}_${t}_$rep.err || { tail -20 $O/b_${lib}_${t}_$rep.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/b_${lib}_${t}_$rep.json').read().strip().splitlines()[-1])
r=d['roofline']; m=d['mnist_as_tf']
print('$lib tile $t rep $rep: convnet %.2f M (net %.3f ms x %d launches, step %.2f ms)  mnist_as_tf %.2f M (step %.2f ms)' % (d['value']/1e6, r['avg_ms'], r['launches'], d['ms_per_step'], m['value']/1e6, m['ms_per_step']))
"
    done
  done
done
echo "== done"
