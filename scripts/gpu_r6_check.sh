#!/bin/bash
# Round-6 kernels on one box: their parity tests, then their timings (scripts/bench_r6_ops.py, bench_sam.py).
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv1x1.py tests/test_gpu_tiled.py \
  -k "lsq or mirror or convex or conv1x1 or interp or softargmin or sam or tile_gather" -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/r6/tests1.log 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_r6_ops.py > gpurun_out/r6/bench_ops.log 2>&1 || exit 1
timeout -k 10 120 python scripts/bench_sam.py > gpurun_out/r6/sam.log 2>&1 || exit 1
