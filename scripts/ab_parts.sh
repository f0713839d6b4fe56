#!/bin/bash
# Interleaved A/B of bench.py schedule overrides (graph replay), two passes on one box; prints the
# headline value of each run.  usage: scripts/ab_parts.sh "opts1" "opts2" ... (empty string = default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
i=0
for pass in 1 2; do
  for o in "$@"; do
    i=$((i + 1))
    if [ -z "$o" ]; then a=""; else a="--opts $o"; fi
    timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-epe $a > gpurun_out/ab/parts_$i.log 2>&1 || exit 1
    v=$(tail -n 1 gpurun_out/ab/parts_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"{d['value']:.2f} pairs/s {d['ms_per_step']:.2f} ms\")")
    echo "pass $pass [${o:-default}]: $v"
  done
done
