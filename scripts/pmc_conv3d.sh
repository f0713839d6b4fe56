# PMC passes over the 3-D split-f16 MFMA conv (conv3d_mfma.hip) at cfg2's final_agg volume (or
# SHAPE=agg16), one rocprofv3 run per pass (MI355X_MICROARCH.md: separate --pmc passes).
# usage (GPU box): SHAPE=final_agg bash scripts/pmc_conv3d.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_c3_${SHAPE:-final_agg}
mkdir -p $OUT
CMD="python3 $R/scripts/bench_conv3d_mf.py 3 --only=${SHAPE:-final_agg}"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex conv3d_mf_kernel -d $OUT/$1 -o $1 --output-format csv -- $CMD > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
run p3 "SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM"
run p4 "FETCH_SIZE"
run p5 "WRITE_SIZE"
python3 $R/scripts/pmc_summary.py $OUT
