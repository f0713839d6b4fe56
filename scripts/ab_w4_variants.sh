#!/bin/bash
# F(4x4) variants against the in-tree library (VARS, default "dup": variants/dup.so built with
# -DSA_W4_DUP=1; "dmaat": -DSA_W4_DMA_AT=1): split-kernel parity tests on each variant, then
# per-conv times (bench_conv2d.py --split --only-wino) and the default bench line, interleaved
# twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
VARS=${VARS:-dup}
for v in $VARS; do
  SA_HIP_LIB=variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_wino.py -k "split or flow_head or wino4" > gpurun_out/ab/${v}_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/ab/${v}_tests.log; [ $rc -eq 0 ] || exit 1
done
for pass in 1 2; do
  for v in tree $VARS; do
    if [ $v = tree ]; then lib=""; else lib="variants/$v.so"; fi
    SA_HIP_LIB=$lib timeout -k 10 200 python scripts/bench_conv2d.py --split --only-wino > gpurun_out/ab/c_${v}_$pass.log 2>&1 || exit 1
    SA_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab/b_${v}_$pass.log 2>&1 || exit 1
  done
done
for v in tree $VARS; do
  echo "== $v"
  for pass in 1 2; do grep "split" gpurun_out/ab/c_${v}_$pass.log | sed 's/^\([a-z0-9.]*\) .*split *\([0-9.]*\) us.*/\1 \2/' | tr '\n' ' '; echo; done
  for pass in 1 2; do tail -n 1 gpurun_out/ab/b_${v}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); r = d["roofline"]
print(d["value"], d["ms_per_step"], "w4", r["ms_per_step"], "epe", d.get("epe_vs_reference"), "redo", d.get("split_redo_blocks"))'; done
done
