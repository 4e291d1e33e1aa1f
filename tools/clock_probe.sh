#!/bin/bash
# Sample the GPU's shader clock and power while the whole-network kernel runs (netbench
# with many repetitions): is the fp64-VALU-bound kernel clock/power limited?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/clock}
mkdir -p $OUT
CFG=${CFG:-mnist_paper_convnet_gp}
timeout -k 10 120 python3 tools/netbench.py --configs $CFG --reps ${REPS:-400} > $OUT/netbench_$CFG.log 2>&1 &
PID=$!
sleep ${DELAY:-12}
for k in 1 2 3; do
  timeout 20 rocm-smi --showclocks --showpower --showtemp > $OUT/smi_${CFG}_$k.txt 2>&1
  sleep 1
done
wait $PID
echo "netbench rc=$?"
cat $OUT/netbench_$CFG.log | grep -v amdgpu.ids
grep -hE "sclk|Power|power|Temperature" $OUT/smi_${CFG}_*.txt | head -20
