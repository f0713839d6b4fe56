#!/bin/bash
# Graph instances in flight (bench.py --pipeline 1 / 2 / 3), interleaved twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
for pass in 1 2; do
  for p in 1 2 3; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --pipeline $p --steps ${STEPS:-10} > gpurun_out/ab/pl_${p}_$pass.log 2>&1 || exit 1
  done
done
for p in 1 2 3; do
  echo "== pipeline $p"
  for pass in 1 2; do tail -n 1 gpurun_out/ab/pl_${p}_$pass.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); r = d["roofline"]
print(d["value"], d["ms_per_step"], "w4", r["ms_per_step"], "epe", d.get("epe_vs_reference"), "graph-eager", d.get("graph_vs_eager_max_abs"), d.get("execution")[:40])'; done
done
