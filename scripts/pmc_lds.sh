# LDS bank-conflict pass of the F(4x4) kernel on one conv shape, for the default build and the
# -DSA_W4_DIAG=7 variant (no filter reads in the main loop).
# usage: SHAPE=xc08 bash scripts/pmc_lds.sh   (variants/diag7.so built beforehand)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=${SHAPE:-xc08}
mkdir -p $R/gpurun_out/pmc_lds
for v in base diag7 diag6; do
  lib=$R/stereoanywhere_amd/lib/libsa_hip.so
  [ $v != base ] && lib=$R/variants/$v.so
  SA_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA \
    --kernel-include-regex wino_f4k3 -d $R/gpurun_out/pmc_lds/$v -o $v --output-format csv -- \
    python3 $R/scripts/bench_conv2d.py --only-wino --shape=$S > $R/gpurun_out/pmc_lds/$v.log 2>&1
done
for v in base diag7 diag6; do echo "== $v"; python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_lds/$v; done
