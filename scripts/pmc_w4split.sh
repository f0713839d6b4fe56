#!/bin/bash
# PMC passes over the split F(4x4) kernel at xc08 (bench_conv2d.py --split runs the fp32 kernel too;
# pmc_summary.py lists both), one rocprofv3 run per pass as MI355X_MICROARCH.md prescribes
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcw
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex wino_f4k3 -d $R/gpurun_out/pmcw/$1 -o $1 --output-format csv -- python3 $R/scripts/bench_conv2d.py --split --shape=${SHAPE:-xc08} > $R/gpurun_out/pmcw/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit 1
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" || exit 1
run p3 "SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM" || exit 1
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmcw > $R/gpurun_out/pmcw/summary.txt
