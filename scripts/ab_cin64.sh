#!/bin/bash
# Round 6: the F(4x4) launches of 64-channel convs on large planes (the feature encoder's layer1,
# 544 x 960) on the fp32-product kernel (bench.py --w4-fp32-cin64 262144) against the split kernel
# everywhere (0), forward lines interleaved three times (the --w4-fp32-cin64 knob measured slower and was
# removed; record: profiles/ab/r06_cin64_large_planes.txt)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/cin64
for pass in 1 2 3; do
  for v in 0 262144; do
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe --w4-fp32-cin64 $v > gpurun_out/cin64/f_${v}_$pass.log 2>&1 || exit 1
    tail -n 1 gpurun_out/cin64/f_${v}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); k = d["roofline"]["kernels"]
print(sys.argv[1], round(d["value"], 2), round(d["ms_per_step"], 2), "w4", round(k["conv2d_wino4"]["ms_per_step"], 2))' "px$v" >> gpurun_out/cin64/summary.txt
  done
done
