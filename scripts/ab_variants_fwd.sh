#!/bin/bash
# Forward A/B of every variants/*.so against the in-tree build: bench.py (no CPU baseline, no
# EPE) interleaved twice; outputs gpurun_out/abv/b_<variant>_<round>.json
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abv
for round in 1 2; do
  for v in in-tree variants/*.so; do
    tag=$(basename $v .so)
    if [ "$v" = in-tree ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-epe > gpurun_out/abv/b_${tag}_$round.json 2>/dev/null || exit 1
    else
      SA_HIP_LIB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-epe > gpurun_out/abv/b_${tag}_$round.json 2>/dev/null || exit 1
    fi
  done
done
