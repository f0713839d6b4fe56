#!/bin/bash
# softargmin_conf A/B (round 6: unconditional clamped loads + the n = 240 instantiation) against a
# comparison build (variants/samhead.so = scripts/build_variant.sh samhead HEAD softargmin.hip):
# the softargmin parity tests on the in-tree build, then scripts/bench_sam.py interleaved twice
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/sam
V=${1:-variants/samhead.so}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py -k "softargmin or sam or forward or epe or reference" \
  > gpurun_out/sam/tests.log 2>&1 || exit 1
for pass in 1 2; do
  for shape in "4 136 240" "25 224 280"; do
    echo "== in-tree $pass $shape" >> gpurun_out/sam/bench.txt
    timeout -k 10 120 python scripts/bench_sam.py $shape >> gpurun_out/sam/bench.txt 2>&1 || exit 1
    echo "== $V $pass $shape" >> gpurun_out/sam/bench.txt
    SA_HIP_LIB=$V timeout -k 10 120 python scripts/bench_sam.py $shape >> gpurun_out/sam/bench.txt 2>&1 || exit 1
  done
done
