#!/bin/bash
# Texture-path occupancy of net_kernel (the variance-map load stream): one rocprofv3 --pmc
# pass per config with the TA / TD busy counters, over one B=1024 Kxz tile x 3
# (tools/netbench.py --reps 1).  Summary: tools/pmc_ta.py -> ta_pmc.json.
#   OUT=gpurun_out/x bash tools/pmc_ta.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_ta}
CFGS=${PMC_CFGS:-"mnist_paper_convnet_gp mnist_as_tf"}
mkdir -p $OUT
for cfg in $CFGS; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum \
        TD_TD_BUSY_sum GRBM_GUI_ACTIVE -f csv -d $OUT/${cfg}_ta -o pmc -- \
        python3 tools/netbench.py --configs $cfg --reps 1 > $OUT/${cfg}_ta.log 2>&1
    rc=$?
    echo "== ${cfg}_ta rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/${cfg}_ta.log; exit $rc; fi
done
python3 tools/pmc_ta.py $OUT
