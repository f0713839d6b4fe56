#!/bin/bash
# Floor of a two-chunks-ahead DMA ring for the split F(4x4) kernel: the
# in-tree library against variants/d9.so (SA_W4_DIAG=9: the loop waits for chunk kc - 1's DMAs
# only; wrong results, timing only), interleaved twice on one box, then PMC passes of both on xc08.
# build: scripts/build_variant.sh d9 WORKTREE conv2d_wino4.hip -fno-slp-vectorize -DSA_W4_DIAG=9
# usage: scripts/diag_ring.sh [times|pmc]
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd "$R"
mkdir -p gpurun_out/ring
S="--split --shape=xc08 --shape=hzr08 --shape=qh08 --shape=mot --shape=fnet.layer1 --shape=xc16 --shape=fnet.layer3"
if [ "${1:-times}" = times ]; then
  for pass in 1 2; do
    echo "== in-tree pass $pass" >> gpurun_out/ring/variants.log
    timeout -k 10 150 python scripts/bench_conv2d.py $S >> gpurun_out/ring/variants.log 2>&1 || exit 1
    echo "== d9 pass $pass" >> gpurun_out/ring/variants.log
    SA_HIP_LIB=variants/d9.so timeout -k 10 150 python scripts/bench_conv2d.py $S >> gpurun_out/ring/variants.log 2>&1 || exit 1
  done
  exit 0
fi
cd /tmp && export TMPDIR=/tmp
run() {   # name, counters, [library]
  SA_HIP_LIB=${3:-} timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-include-regex wino_f4k3 -d $R/gpurun_out/ring/pmc_$1 -o $1 \
    --output-format csv -- python3 $R/scripts/bench_conv2d.py --split --shape=xc08 > $R/gpurun_out/ring/pmc_$1.log 2>&1
}
for v in base d9; do
  lib=""; [ $v = d9 ] && lib=$R/variants/d9.so
  run ${v}_p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" $lib || exit 1
  run ${v}_p2 "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" $lib || exit 1
done
