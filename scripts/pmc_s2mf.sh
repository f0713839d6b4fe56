# PMC passes over the stride-2 16 -> 32 MFMA conv (conv3d_s2mf_kernel) at cfg2's gated volume
# (scripts/bench_s2mf.py 0), one rocprofv3 run per pass (MI355X_MICROARCH.md).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_s2
mkdir -p $OUT
CMD="python3 $R/scripts/bench_s2mf.py 0"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex "conv3d_s2mf_kernel" -d $OUT/$1 -o $1 --output-format csv -- $CMD > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM"
run p3 "FETCH_SIZE"
run p4 "WRITE_SIZE"
python3 $R/scripts/pmc_summary.py $OUT
