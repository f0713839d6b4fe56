#!/bin/bash
# Round-6 second pass: the corr split + convex / LSQ changes' tests, the model tests, then one bench.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -k "corr or lsq or convex or shear or lookup" -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/r6/tests2.log 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_r6_ops.py > gpurun_out/r6/bench_ops2.log 2>&1 || exit 1
timeout -k 10 100 python scripts/bench_corr.py > gpurun_out/r6/corr.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r6/model.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r6/bench.log 2>&1 || exit 1
