#!/bin/bash
# GPU ops tests + the default and cfg5 bench lines, with a one-line summary of each
# (value, ms/step, gru_plumbing and misc ms/step, F(4x4) ms/step, EPE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests 2>&1 | tail -3 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/b_default.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config cfg5 --no-cpu-baseline > gpurun_out/b_cfg5.log 2>&1 || exit 1
for f in gpurun_out/b_default.log gpurun_out/b_cfg5.log; do
  tail -n 1 "$f" | python -c '
import sys, json
d = json.loads(sys.stdin.read()); r = d["roofline"]
print(d["value"], d["ms_per_step"], "plumb", r["kernels"]["gru_plumbing"]["ms_per_step"], "misc",
      r.get("misc_ms_per_step"), "w4", r["ms_per_step"], "epe", d.get("epe_vs_reference"))'
done
