#!/bin/bash
# softargmin_conf A/B (round 6: unconditional clamped loads + the n = 240 instantiation) against a
# comparison build (variants/samhead.so = scripts/build_variant.sh samhead HEAD softargmin.hip):
# the softargmin parity tests on the in-tree build, then scripts/bench_sam.py interleaved twice
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/sam
V=${1:-variants/samhead.so}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "softargmin or sam" \
  > gpurun_out/sam/tests.log 2>&1 || exit 1
for pass in 1 2; do
  echo "== in-tree $pass" >> gpurun_out/sam/bench.txt
  timeout -k 10 120 python scripts/bench_sam.py >> gpurun_out/sam/bench.txt 2>&1 || exit 1
  echo "== $V $pass" >> gpurun_out/sam/bench.txt
  SA_HIP_LIB=$V timeout -k 10 120 python scripts/bench_sam.py >> gpurun_out/sam/bench.txt 2>&1 || exit 1
done
# the F(4x4) prologue with kernel arguments in device memory (first DMA ~2.8k cycles after start)
if [ -f variants/clock.so ]; then
  SA_HIP_LIB=variants/clock.so timeout -k 10 120 python scripts/w4_clock.py 4 128 128 136 240 > gpurun_out/sam/kernarg.txt 2>&1 || exit 1
  HIP_FORCE_DEV_KERNARG=1 SA_HIP_LIB=variants/clock.so timeout -k 10 120 python scripts/w4_clock.py 4 128 128 136 240 >> gpurun_out/sam/kernarg.txt 2>&1 || exit 1
  HIP_FORCE_DEV_KERNARG=0 SA_HIP_LIB=variants/clock.so timeout -k 10 120 python scripts/w4_clock.py 4 128 128 136 240 >> gpurun_out/sam/kernarg.txt 2>&1 || exit 1
fi
