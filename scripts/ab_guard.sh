#!/bin/bash
# A/B of the split kernels (the in-tree library, with the f16 range guard) against round 3's library
# (variants/r3.so), per conv: F(4x4) (scripts/bench_conv2d.py --split --only-wino) and the direct
# convs (scripts/bench_direct.py --split), interleaved twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
VARS=${VARS:-"tree r3"}
for pass in 1 2; do
  for v in $VARS; do
    if [ $v = tree ]; then lib=""; else lib="variants/$v.so"; fi
    SA_HIP_LIB=$lib timeout -k 10 200 python scripts/bench_conv2d.py --split --only-wino > gpurun_out/ab/${v}_$pass.log 2>&1 || exit 1
    SA_HIP_LIB=$lib timeout -k 10 200 python scripts/bench_direct.py --split > gpurun_out/ab/${v}_d$pass.log 2>&1 || exit 1
  done
done
for v in $VARS; do
  echo "== $v"; for pass in 1 2; do grep "split" gpurun_out/ab/${v}_$pass.log | sed 's/^\([a-z0-9.]*\) .*split *\([0-9.]*\) us.*/\1 \2/' | tr '\n' ' '; echo; done
  for pass in 1 2; do grep "split" gpurun_out/ab/${v}_d$pass.log | sed 's/^\([a-z0-9.]*\) .*split *\([0-9.]*\) us.*/\1 \2/' | tr '\n' ' '; echo; done
done
