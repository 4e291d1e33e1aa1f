set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r5l; mkdir -p $OUT
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"
for cfg in mnist_paper_convnet_gp mnist_as_tf; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ -f csv -d $OUT/${cfg}_sq -o pmc -- python3 tools/netbench.py --configs $cfg --reps 1 --dtype f32 > $OUT/${cfg}_sq.log 2>&1 || { echo fail $cfg sq; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -f csv -d $OUT/${cfg}_ta -o pmc -- python3 tools/netbench.py --configs $cfg --reps 1 --dtype f32 > $OUT/${cfg}_ta.log 2>&1 || { echo fail $cfg ta; exit 1; }
  echo "== $cfg done"
done
python3 tools/pmc_ta.py $OUT > /dev/null
