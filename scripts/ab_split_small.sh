#!/bin/bash
# The 4-wave split shape (ops.W4_SPLIT_SMALL_CIN, block_shape 7) for launches with Cin <= 64 /
# 128 / all, against the default: its parity tests, per-conv times, then the default bench line
# interleaved twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino.py \
  tests/test_gpu_model.py -k "small or range_guard" > gpurun_out/ab/ss_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/ss_tests.log; [ $rc -eq 0 ] || exit 1
for pass in 1 2; do
  for c in 0 64 128 4096; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --w4-split-small-cin $c > gpurun_out/ab/ss_${c}_$pass.log 2>&1 || exit 1
  done
done
for c in 0 64 128 4096; do
  echo "== Cin <= $c"
  for pass in 1 2; do tail -n 1 gpurun_out/ab/ss_${c}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); r = d["roofline"]
print(d["value"], d["ms_per_step"], "w4", r["ms_per_step"], "epe", d.get("epe_vs_reference"), "redo", d.get("split_redo_blocks"))'; done
done
