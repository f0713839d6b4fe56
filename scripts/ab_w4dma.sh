#!/bin/bash
# Round 6: the paired split F(4x4) loop against the DMA-wait floor (variants/d9.so, SA_W4_DIAG=9:
# waits for chunk kc - 1's DMAs only, wrong results) and the next chunk's DMA issued all at
# column 0 (variants/early.so, SA_W4_DMA_EARLY=1): per-conv times (bench_conv2d.py --split),
# interleaved twice, then forward lines of the in-tree build and early.so (the SA_W4_DMA_EARLY switch
# was measured slower and removed: profiles/ab/r06_w4_dma_floor.txt)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/w4dma
for pass in 1 2; do
  for v in in-tree variants/d9.so variants/early.so; do
    echo "== $v $pass" >> gpurun_out/w4dma/conv.txt
    if [ "$v" = in-tree ]; then
      timeout -k 10 300 python scripts/bench_conv2d.py --split >> gpurun_out/w4dma/conv.txt 2>&1 || exit 1
    else
      SA_HIP_LIB=$v timeout -k 10 300 python scripts/bench_conv2d.py --split >> gpurun_out/w4dma/conv.txt 2>&1 || exit 1
    fi
  done
done
for pass in 1 2; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe > gpurun_out/w4dma/fwd_intree_$pass.log 2>&1 || exit 1
  SA_HIP_LIB=variants/early.so timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-epe > gpurun_out/w4dma/fwd_early_$pass.log 2>&1 || exit 1
done
