#!/bin/bash
# Round 6 (late): the same-box check of the wave-priority flag: the built library (conv2d_wino4 with
# -mllvm -amdgpu-set-wave-priority) against variants/w4noprio.so (without it), forward lines
# interleaved three times
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/w4q
V=${1:-variants/w4noprio.so}
for pass in 1 2 3; do
  for v in built variant; do
    if [ $v = variant ]; then export SA_HIP_LIB=$V; else unset SA_HIP_LIB; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe > gpurun_out/w4q/f_${v}_$pass.log 2>&1 || exit 1
    tail -n 1 gpurun_out/w4q/f_${v}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); k = d["roofline"]["kernels"]
print(sys.argv[1], round(d["value"], 2), round(d["ms_per_step"], 2), "w4", round(k["conv2d_wino4"]["ms_per_step"], 2), "one-stream", round(d["roofline"]["one_stream_ms_per_step"], 2))' "$v" >> gpurun_out/w4q/summary.txt
  done
done
