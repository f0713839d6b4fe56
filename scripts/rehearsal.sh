#!/bin/bash
# Rehearsal of the driver's round-end GPU commands on a fresh box: pytest -m gpu, smoke(), the
# default bench line; each step under its own time limit (gpu_steps.sh), outputs under
# gpurun_out/rehearsal.  A summary goes to gpurun_out/rehearsal/summary.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
mkdir -p gpurun_out/rehearsal
steps=(
  "rh_tests:900:python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread"
  "rh_smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
  "rh_bench:420:python bench.py"
)
bash "$R/scripts/gpu_steps.sh" "${steps[@]}"
rc=$?
{
  echo "## pytest -m gpu"; grep -E "passed|failed" gpurun_out/rh_tests.log | tail -1
  echo "## smoke()"; grep -E "smoke" gpurun_out/rh_smoke.log
  echo "## bench.py (default)"; tail -n 1 gpurun_out/rh_bench.log
} > gpurun_out/rehearsal/summary.txt 2>&1
exit $rc
