#!/bin/bash
# Phase clocks of the F(4x4) split kernel (scripts/w4_clock.py) on the model's shapes for each clock
# build given (default variants/clock.so = scripts/build_variant.sh clock WORKTREE conv2d_wino4.hip
# -fno-slp-vectorize -DSA_W4_CLOCK; diagnostic builds add -DSA_W4_DIAG=n)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/clk
libs=("$@")
[ ${#libs[@]} -eq 0 ] && libs=(variants/clock.so)
for lib in "${libs[@]}"; do
  for s in "4 256 384 136 240" "4 128 128 136 240" "8 64 64 544 960"; do
    echo "== $lib $s" >> gpurun_out/clk/clock.txt
    SA_HIP_LIB=$lib timeout -k 10 120 python scripts/w4_clock.py $s >> gpurun_out/clk/clock.txt 2>&1 || exit 1
  done
done
