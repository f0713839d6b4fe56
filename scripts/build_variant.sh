#!/bin/bash
# Build an alternative libsa_hip.so into variants/<name>.so with one source file taken from
# a git revision (A/B timing on the same box: SA_HIP_LIB=variants/<name>.so).
# usage: scripts/build_variant.sh <name> <rev|WORKTREE> <csrc file name> [extra hipcc flags...]
set -euo pipefail
name=$1 rev=$2 file=$3
shift 3
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
cp "$root"/build/*.o "$tmp"/
if [ "$rev" = WORKTREE ]; then
  cp "$root/stereoanywhere_amd/csrc/$file" "$tmp/$file"
else
  git -C "$root" show "$rev:stereoanywhere_amd/csrc/$file" > "$tmp/$file"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result \
  -I "$root/stereoanywhere_amd/csrc" "$@" -c "$tmp/$file" -o "$tmp/${file%.hip}.o"
mkdir -p "$root/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/variants/$name.so" "$tmp"/*.o
rm -rf "$tmp"
echo "built variants/$name.so"
