# HBM traffic of the GRU loop's lookup (+ convc1) in the cfg2 forward: rocprofv3 FETCH_SIZE and
# WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md) over a one-stream eager bench (whole
# batch per launch), summarised per kernel.  usage (GPU box): bash scripts/pmc_lookup_model.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_lkm
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "lookup_c1|corr_pyramid_v2|pyramid_from_strided" -d $OUT/$c -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-epe --no-graph --one-stream > $OUT/$c.log 2>&1
done
python3 $R/scripts/pmc_summary.py $OUT
