#!/bin/bash
# Split-kernel diagnostics on one box: MFMA issue rates, the SA_W4_DIAG variants (variants/d*.so)
# of bench_conv2d.py --split, and PMC passes over the split and fp32 F(4x4) kernels.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/diag
timeout -k 10 60 ./scripts/micro/mfma_rate > gpurun_out/diag/mfma_rate.log 2>&1 || exit 1
for v in in-tree variants/d2.so variants/d3.so variants/d5.so variants/d8.so; do
  echo "== $v" >> gpurun_out/diag/variants.log
  if [ "$v" = in-tree ]; then
    timeout -k 10 120 python scripts/bench_conv2d.py --split --shape=xc08 --shape=hzr08 --shape=fnet.layer1 >> gpurun_out/diag/variants.log 2>&1 || exit 1
  else
    SA_HIP_LIB=$v timeout -k 10 120 python scripts/bench_conv2d.py --split --shape=xc08 --shape=hzr08 --shape=fnet.layer1 >> gpurun_out/diag/variants.log 2>&1 || exit 1
  fi
done
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex wino_f4k3 -d $R/gpurun_out/diag/pmc_$1 -o $1 --output-format csv -- python3 $R/scripts/bench_conv2d.py --split --shape=xc08 > $R/gpurun_out/diag/pmc_$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit 1
run p2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" || exit 1
run p3 "SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM" || exit 1
