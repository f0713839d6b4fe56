# PMC passes over the fused lookup + convc1 (row layout: lookup_c1_vec_kernel; sheared:
# lookup_c1_shear_kernel) at cfg2's shape, one rocprofv3 run per pass (MI355X_MICROARCH.md).
# usage (GPU box): SHAPE=cfg2 bash scripts/pmc_lookup.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_lk_${SHAPE:-cfg2}
mkdir -p $OUT
CMD="python3 $R/scripts/bench_shear.py --shape=${SHAPE:-cfg2} --only=lookup --reps=3"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex lookup_c1 -d $OUT/$1 -o $1 --output-format csv -- $CMD > $OUT/$1.log 2>&1
}
run p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE"
run p2 "FETCH_SIZE"
run p3 "WRITE_SIZE"
run p4 "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
run p5 "TA_FLAT_WRITE_WAVEFRONTS_sum TA_BUSY_max TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum"
python3 $R/scripts/pmc_summary.py $OUT
