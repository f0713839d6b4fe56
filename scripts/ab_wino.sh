#!/bin/bash
# A/B the Winograd convs: every variants/*.so vs the in-tree build, interleaved twice
# usage: scripts/ab_wino.sh [bench_conv2d.py args...]
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
for round in 1 2; do
  for v in variants/*.so in-tree; do
    echo "== $v (round $round)"
    if [ "$v" = in-tree ]; then
      timeout -k 10 300 python scripts/bench_conv2d.py --only-wino "$@" || exit 1
    else
      SA_HIP_LIB=$v timeout -k 10 300 python scripts/bench_conv2d.py --only-wino "$@" || exit 1
    fi
  done
done
