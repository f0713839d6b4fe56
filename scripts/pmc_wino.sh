set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex wino_f2k3 -d $R/gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 $R/scripts/bench_conv2d.py --only-wino --shape=xc08
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC --kernel-include-regex wino_f2k3 -d $R/gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 $R/scripts/bench_conv2d.py --only-wino --shape=xc08
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL --kernel-include-regex wino_f2k3 -d $R/gpurun_out/pmc/p3 -o p3 --output-format csv -- python3 $R/scripts/bench_conv2d.py --only-wino --shape=xc08 || echo "p3 failed"
find $R/gpurun_out/pmc -name "*counter_collection*" | head
