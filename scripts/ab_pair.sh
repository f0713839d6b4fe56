#!/bin/bash
# A/B of a split F(4x4) kernel change (round 6: the paired-channel MFMA loop, SA_W4_PAIR, and its
# job-innermost filter layout) against a comparison build of conv2d_wino4.hip (e.g.
# scripts/build_variant.sh head HEAD conv2d_wino4.hip -fno-slp-vectorize, or WORKTREE with
# -DSA_W4_PAIR=0): the wino parity tests on the in-tree build, then per-conv times and two
# interleaved passes of short bench lines.  usage: scripts/ab_pair.sh [variants/<name>.so]
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pair
V=${1:-variants/head.so}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wino.py \
  > gpurun_out/pair/tests.log 2>&1 || exit 1
for pass in 1 2; do
  for v in in-tree "$V"; do
    echo "== $v pass $pass" >> gpurun_out/pair/conv.txt
    if [ "$v" = in-tree ]; then
      timeout -k 10 300 python scripts/bench_conv2d.py --split >> gpurun_out/pair/conv.txt 2>&1 || exit 1
    else
      SA_HIP_LIB=$v timeout -k 10 300 python scripts/bench_conv2d.py --split >> gpurun_out/pair/conv.txt 2>&1 || exit 1
    fi
  done
done
B="python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe"
run() {   # name, library ("" = in-tree)
  if [ -n "$2" ]; then
    SA_HIP_LIB=$2 timeout -k 10 240 $B > gpurun_out/pair/$1.log 2>&1 || exit 1
  else
    timeout -k 10 240 $B > gpurun_out/pair/$1.log 2>&1 || exit 1
  fi
  tail -n 1 gpurun_out/pair/$1.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); k = d["roofline"]["kernels"]
print(sys.argv[1], round(d["value"], 2), round(d["ms_per_step"], 2), "w4", round(k["conv2d_wino4"]["ms_per_step"], 2))' "$1" \
    >> gpurun_out/pair/summary.txt
}
for pass in 1 2; do
  run pair1_$pass ""
  run variant_$pass "$V"
done
