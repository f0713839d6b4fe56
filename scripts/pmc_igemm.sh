# PMC passes over the implicit-GEMM conv (conv2d_igemm.hip) on one model shape (default zr08), one
# rocprofv3 run per pass (MI355X_MICROARCH.md: separate --pmc passes, no tracing beside them).
# usage (GPU box): SHAPE=zr08 bash scripts/pmc_igemm.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_ig_${SHAPE:-zr08}
mkdir -p $OUT
CMD="python3 $R/scripts/bench_igemm.py 5 --only=${SHAPE:-zr08}"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex ig_kernel -d $OUT/$1 -o $1 --output-format csv -- $CMD > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
run p3 "SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM"
python3 $R/scripts/pmc_summary.py $OUT
