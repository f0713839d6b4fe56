#!/bin/bash
# The wall-clock checks (tests/test_perf_gpu.py, marker perf) that the parity gates deselect.
# usage (GPU box): scripts/perf_checks.sh [extra pytest args]
set -uo pipefail
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests/test_perf_gpu.py --run-perf -m perf -v -s --timeout 300 --timeout-method thread "$@"
