#!/bin/bash
# Round 6 (late): the wave-priority pass's VALU threshold on conv2d_wino4 (the LLVM default 100 in
# the built library; variants/w4t40.so, variants/w4t300.so): forward lines interleaved twice, then
# the chosen variant's tests are run separately
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/w4t
for pass in 1 2; do
  for v in built w4t40 w4t300; do
    if [ $v = built ]; then unset SA_HIP_LIB; else export SA_HIP_LIB=variants/$v.so; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe > gpurun_out/w4t/f_${v}_$pass.log 2>&1 || exit 1
    tail -n 1 gpurun_out/w4t/f_${v}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); k = d["roofline"]["kernels"]
print(sys.argv[1], round(d["value"], 2), round(d["ms_per_step"], 2), "w4", round(k["conv2d_wino4"]["ms_per_step"], 2), "one-stream", round(d["roofline"]["one_stream_ms_per_step"], 2))' "$v" >> gpurun_out/w4t/summary.txt
  done
done
