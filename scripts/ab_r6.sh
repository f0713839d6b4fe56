#!/bin/bash
# Round-6 forward-level A/B on one box, two interleaved passes of short bench lines (configs[1],
# no CPU baseline / EPE): the default against each round-6 switch turned back, and the F(4x4)
# Cin <= 64 fp32 knob.  One summary line per run: value, ms/step, conv2d_wino4 ms/step.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab6
B="python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe"
run() {   # name, extra flags
  timeout -k 10 240 $B $2 > gpurun_out/ab6/$1.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab6/$1.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); k = d["roofline"]["kernels"]
print(sys.argv[1], round(d["value"], 2), round(d["ms_per_step"], 2), "w4", round(k["conv2d_wino4"]["ms_per_step"], 2),
      "corr", round(k.get("corr_volume_pyramid", {}).get("avg_launch_us", 0), 1))' "$1" >> gpurun_out/ab6/summary.txt
}
for pass in 1 2; do
  run default$pass ""
  run directsmall0_$pass "--direct-small 0"
  run conv1x1off_$pass "--conv1x1 0"
done
