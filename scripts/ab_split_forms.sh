#!/bin/bash
# A/B of the split kernel's forms in the forward: the in-tree build (W4S_K32 default) against
# variants/k2.so (paired) and variants/k3.so (paired, staged rows): bench.py headline (no CPU
# baseline, no EPE) and the per-launch anatomy, interleaved twice.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for round in 1 2; do
  for v in in-tree variants/k2.so variants/k3.so; do
    tag=$(basename $v .so)
    if [ "$v" = in-tree ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-epe > gpurun_out/ab/b_${tag}_$round.json 2>/dev/null || exit 1
    else
      SA_HIP_LIB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-epe > gpurun_out/ab/b_${tag}_$round.json 2>/dev/null || exit 1
    fi
  done
done
for v in in-tree variants/k2.so variants/k3.so; do
  tag=$(basename $v .so)
  if [ "$v" = in-tree ]; then
    timeout -k 10 300 python scripts/wino4_launches.py > gpurun_out/ab/wl_$tag.log 2>&1 || exit 1
  else
    SA_HIP_LIB=$v timeout -k 10 300 python scripts/wino4_launches.py > gpurun_out/ab/wl_$tag.log 2>&1 || exit 1
  fi
done
