#!/usr/bin/env python3
"""Shader clock held by the F(4x4) Winograd conv: runs one conv shape of bench_conv2d.py with a
library built with -DSA_W4_CLOCK (SA_HIP_LIB=variants/clock.so) and reads every block's
(s_memtime, s_memrealtime) stamps: clock = d(memtime) / d(memrealtime) x 100 MHz."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import _native as N, ops  # noqa: E402

N_, Cin, Cout, H, W = 4, 256, 384, 136, 240
if len(sys.argv) > 1:
    N_, Cin, Cout, H, W = map(int, sys.argv[1:6])
x = torch.randn(N_, Cin, H, W, device="cuda")
w = torch.randn(Cout, Cin, 3, 3, device="cuda") / (3 * Cin ** 0.5)
U = ops.wino_weights(w)
for _ in range(20):
    ops.conv2d_k3(x, U)
torch.cuda.synchronize()
nb = ops._wino4_blocks(x, U)
fn = N.lib().sa_w4_clock_read
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((min(nb, 65536), 12), dtype=np.uint64)
assert fn(buf.ctypes.data, buf.shape[0]) == 0
d_t = (buf[:, 2] - buf[:, 0]).astype(np.float64)
d_r = (buf[:, 3] - buf[:, 1]).astype(np.float64)
clk = d_t / d_r * 100.0   # MHz
print(f"{nb} blocks: clock median {np.median(clk):.0f} MHz (p10 {np.percentile(clk, 10):.0f}, p90 "
      f"{np.percentile(clk, 90):.0f}); block duration median {np.median(d_r) / 100:.1f} us, "
      f"{np.median(d_t):.0f} cycles: first chunk landed after {np.median(buf[:, 4] - buf[:, 0]):.0f}, main loop "
      f"{np.median(buf[:, 5] - buf[:, 4]):.0f}, epilogue {np.median(buf[:, 2] - buf[:, 5]):.0f} (transform + exchange "
      f"{np.median(buf[:, 6] - buf[:, 5]):.0f}, barrier + stats {np.median(buf[:, 7] - buf[:, 6]):.0f}, stores "
      f"{np.median(buf[:, 2] - buf[:, 7]):.0f}); first chunk: last wave started at "
      f"{np.median(buf[:, 9].astype(np.int64) - buf[:, 0].astype(np.int64)):.0f}, wave 0 issued it at "
      f"{np.median(buf[:, 8] - buf[:, 0]):.0f} (item decoded at {np.median(buf[:, 10] - buf[:, 0]):.0f}, chunk 0's filter DMA "
      f"issued at {np.median(buf[:, 11] - buf[:, 0]):.0f})")
