#!/bin/bash
# HIP hardware queues per process (GPU_MAX_HW_QUEUES 4 = the box default, 8, 16) for the default
# schedule and for two / three forwards in flight (bench.py --pipeline), interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
for pass in 1 2; do
  for q in 4 8 16; do
    for p in 1 2 3; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --no-epe --pipeline $p --steps 10 \
        > gpurun_out/ab/hq_${q}_${p}_$pass.log 2>&1 || exit 1
    done
  done
done
for q in 4 8 16; do
  for p in 1 2 3; do
    echo "== queues $q pipeline $p"
    for pass in 1 2; do
      grep -ho "execution probe: graph [0-9.]* ms, eager [0-9.]* ms" gpurun_out/ab/hq_${q}_${p}_$pass.log
      tail -n 1 gpurun_out/ab/hq_${q}_${p}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read())
print(d["value"], d["ms_per_step"], d.get("execution")[:30])'
    done
  done
done
