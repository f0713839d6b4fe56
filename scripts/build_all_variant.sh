#!/bin/bash
# Build an alternative libsa_hip.so into variants/<name>.so with extra hipcc flags on EVERY source
# (the Makefile's per-file flags kept): A/B of a compiler option across the library.
# usage: scripts/build_all_variant.sh <name> [extra hipcc flags...]
set -euo pipefail
name=$1
shift 1
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
for f in "$root"/stereoanywhere_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  extra=()
  [ "$b" = conv2d_wino4 ] && extra=(-fno-slp-vectorize -mllvm -amdgpu-set-wave-priority)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result \
    -I "$root/stereoanywhere_amd/csrc" "${extra[@]}" "$@" -c "$f" -o "$tmp/$b.o" &
  while [ "$(jobs -r | wc -l)" -ge 6 ]; do sleep 1; done
done
wait
mkdir -p "$root/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/variants/$name.so" "$tmp"/*.o
rm -rf "$tmp"
echo "built variants/$name.so"
