# PMC passes (one rocprofv3 run each, as MI355X_MICROARCH.md prescribes) over one conv shape of
# scripts/bench_conv2d.py.  usage: KREGEX=wino_f4k3 SHAPE=xc08 bash scripts/pmc_wino.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K=${KREGEX:-wino_f2k3}
S=${SHAPE:-xc08}
mkdir -p $R/gpurun_out/pmc
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex $K -d $R/gpurun_out/pmc/$1 -o $1 --output-format csv -- python3 $R/scripts/bench_conv2d.py --only-wino --shape=$S > $R/gpurun_out/pmc/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
run p3 "SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM"
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc
