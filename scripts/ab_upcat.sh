#!/bin/bash
# Up-cat pointwise kernel D-tiles per block (in-tree UPCAT_NDT=4 against variants/ndt1.so = the
# round-3 one tile and ndt2.so): hourglass parity tests on each, then the standalone hourglass
# (scripts/bench_hourglass.py) interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py \
  -k "hourglass or upcat or conv3d" > gpurun_out/ab/uc_tests.log 2>&1
rc=$?; tail -1 gpurun_out/ab/uc_tests.log; [ $rc -eq 0 ] || exit 1
for pass in 1 2; do
  for v in tree ndt1 ndt2; do
    if [ $v = tree ]; then lib=""; else lib="variants/$v.so"; fi
    SA_HIP_LIB=$lib timeout -k 10 200 python scripts/bench_hourglass.py 10 > gpurun_out/ab/uc_${v}_$pass.log 2>&1 || exit 1
  done
done
for v in tree ndt1 ndt2; do echo "== $v"; for pass in 1 2; do tail -n 4 gpurun_out/ab/uc_${v}_$pass.log; done; done
