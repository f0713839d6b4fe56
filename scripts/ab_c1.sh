#!/bin/bash
# Round 6: sa_conv1x1's all-channel form (conv1x1_v2_kernel, SA_C1_V2=1, the built library) against
# the round-5 64-channel-block form (variants/c1v1.so, built with -DSA_C1_V2=0): the conv1x1 parity
# tests, the op lines at configs[1]'s sizes and forward lines interleaved twice
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/c1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_model.py -k "conv1x1 or forward or epe" > gpurun_out/c1/tests.log 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_r6_ops.py > gpurun_out/c1/ops_v2.log 2>&1 || exit 1
SA_HIP_LIB=variants/c1v1.so timeout -k 10 200 python scripts/bench_r6_ops.py > gpurun_out/c1/ops_v1.log 2>&1 || exit 1
for pass in 1 2; do
  for v in v2 v1; do
    if [ $v = v1 ]; then export SA_HIP_LIB=variants/c1v1.so; else unset SA_HIP_LIB; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe > gpurun_out/c1/f_${v}_$pass.log 2>&1 || exit 1
    tail -n 1 gpurun_out/c1/f_${v}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); k = d["roofline"]["kernels"]
print(sys.argv[1], round(d["value"], 2), round(d["ms_per_step"], 2), {n: round(v["ms_per_step"], 3) for n, v in k.items() if "1x1" in n or "conv1" in n})' "$v" >> gpurun_out/c1/summary.txt
  done
done
