#!/bin/bash
# Build the whole libsa_hip.so of a git revision into variants/<name>.so (same-box A/B of
# the current Python against an older kernel library: SA_HIP_LIB=variants/<name>.so).
# usage: scripts/build_lib_at.sh <rev> <name>
set -euo pipefail
rev=$1 name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" Makefile include stereoanywhere_amd/csrc | tar -x -C "$tmp"
make -C "$tmp" -j8 >/dev/null
mkdir -p "$root/variants"
cp "$tmp/stereoanywhere_amd/lib/libsa_hip.so" "$root/variants/$name.so"
rm -rf "$tmp"
echo "built variants/$name.so"
