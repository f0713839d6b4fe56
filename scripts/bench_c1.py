#!/usr/bin/env python3
"""sa_conv1x1 at the model's two shapes (configs[1]: 1/4 resolution 136 x 240), HIP events per call
(A/B of library variants: SA_HIP_LIB)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv2d import timeit  # noqa: E402

H4, W4 = 136, 240
tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("SA_HIP_LIB", "built")
for (nb, cin, cout, sc) in ((8, 128, 256, 1.0), (4, 256, 576, 0.25)):
    x = torch.randn(nb, cin, H4, W4, device="cuda")
    w = torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5
    bias = torch.randn(cout, device="cuda")
    ws = ops.conv1x1_weights(w)
    t = timeit(lambda: ops.conv1x1(x, ws, cout, bias, sc), 30)
    nbytes = 4.0 * nb * (cin + cout) * H4 * W4
    print(f"{tag} conv1x1 {nb}x{cin}->{cout}: {t:.1f} us ({nbytes / t / 1e3:.0f} GB/s)")
