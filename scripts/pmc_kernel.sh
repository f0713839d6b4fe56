# PMC passes (one rocprofv3 run each, MI355X_MICROARCH.md) over the kernels matching KREGEX in
# the command CMD (default: the hourglass benchmark).  usage: KREGEX=conv3d_wd bash scripts/pmc_kernel.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K=${KREGEX:-conv3d_wd}
CMD=${CMD:-"python3 $R/scripts/bench_hourglass.py 2"}
OUT=$R/gpurun_out/pmc_${TAG:-k}
mkdir -p $OUT
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex $K -d $OUT/$1 -o $1 --output-format csv -- $CMD > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
run p3 "SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_MFMA"
python3 $R/scripts/pmc_summary.py $OUT
