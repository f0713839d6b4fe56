#!/usr/bin/env python3
"""Phase times of the one-launch weighted LSQ (block 0) from a -DSA_LSQ_CLOCK build:
scripts/build_variant.sh lsqclk WORKTREE lsq.hip -DSA_LSQ_CLOCK; SA_HIP_LIB=variants/lsqclk.so."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import _native as N, ops  # noqa: E402

n = 2 * 136 * 240
for B, spread in ((4, 1.0), (4, 0.01)):
    g = torch.Generator(device="cuda").manual_seed(0)
    m = torch.rand(B, n, device="cuda", generator=g)
    d = (40 * m + 3) * spread + 5 + torch.randn(B, n, device="cuda", generator=g) * spread
    c = torch.rand(B, n, device="cuda", generator=g)
    for _ in range(3):
        ops.weighted_lsq(m, d, c, single_block=True)
    torch.cuda.synchronize()
    buf = (ctypes.c_longlong * 8)()
    N.lib().sa_lsq_clock_read(buf)
    v = list(buf)
    names = ["start", "zeroed", "A hist", "bins found", "B append", "C select", "quantiles", "sums"]
    order = [7, 0, 1, 2, 3, 4, 5, 6]
    t0 = v[7]
    print(f"B={B} spread={spread}: " + ", ".join(f"{names[k]} {(v[i] - t0) / 100:.1f} us" for k, i in enumerate(order)))
