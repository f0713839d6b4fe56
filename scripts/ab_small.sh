#!/bin/bash
# A/B the small update-loop kernels: variants/*.so vs the in-tree build, twice
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
for round in 1 2; do
  for v in variants/*.so in-tree; do
    echo "== $v (round $round)"
    if [ "$v" = in-tree ]; then
      timeout -k 10 300 python scripts/bench_small.py || exit 1
    else
      SA_HIP_LIB=$v timeout -k 10 300 python scripts/bench_small.py || exit 1
    fi
  done
done
