# PMC passes over the hourglass's up-cat pointwise convs (pointwise_upcat_kernel) and the stride-2
# 16 -> 32 conv (conv3d_kernel) at cfg2's volumes (scripts/bench_hourglass.py), one rocprofv3 run
# per pass (MI355X_MICROARCH.md).  usage (GPU box): bash scripts/pmc_upcat.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_up
mkdir -p $OUT
CMD="python3 $R/scripts/bench_hourglass.py 2"
run() {
  timeout -s KILL 150 rocprofv3 --pmc $2 --kernel-include-regex "pointwise_upcat|conv3d_kernel" -d $OUT/$1 -o $1 --output-format csv -- $CMD > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM"
run p3 "FETCH_SIZE"
run p4 "WRITE_SIZE"
python3 $R/scripts/pmc_summary.py $OUT
