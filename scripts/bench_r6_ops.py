#!/usr/bin/env python3
"""Round-6 kernels at configs[1]'s sizes, HIP events per call: the one-launch weighted LSQ (and the
round-5 four-launch form), the convex upsampling, the 1x1 convs (sa_conv1x1 vs F.conv2d / rocBLAS)
and the guidance-pyramid resample (sa_resample_multi vs F.interpolate)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv2d import timeit  # noqa: E402

dev = "cuda"
B, H4, W4 = 4, 136, 240
g = torch.Generator(device="cuda").manual_seed(0)
n = 2 * H4 * W4
m = torch.rand(B, n, device=dev, generator=g)
d = (40 * m + 3) + 5 + torch.randn(B, n, device=dev, generator=g)
c = torch.rand(B, n, device=dev, generator=g)
dz = d.clone()
dz[:, : n // 2] = -1.0   # half the keys relu'd to 0 (the model's synthetic-weight disparities)
dz = dz[:, torch.randperm(n, device=dev, generator=g)].contiguous()
for dd, what in ((d, "positive keys"), (dz, "half zeros")):
    for sb, name in ((True, "one launch"), (False, "round-5 grid form")):
        print(f"weighted_lsq B={B} n={n} {what} {name}: "
              f"{timeit(lambda: ops.weighted_lsq(m, dd, c, single_block=sb), 20):.1f} us")
flow = torch.randn(B, 1, H4, W4, device=dev) * 5
mask = torch.randn(B, 144, H4, W4, device=dev)
t = timeit(lambda: ops.convex_upsample(flow, mask, 4), 20)
nbytes = 4.0 * B * H4 * W4 * (144 + 1 + 16)
print(f"convex_upsample: {t:.1f} us, {nbytes / t / 1e3:.0f} GB/s of {nbytes / 1e6:.1f} MB")
for (nb, cin, cout, sc) in ((8, 128, 256, 1.0), (4, 256, 576, 0.25)):
    x = torch.randn(nb, cin, H4, W4, device=dev)
    w = torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5
    bias = torch.randn(cout, device=dev)
    ws = ops.conv1x1_weights(w)
    t_h = timeit(lambda: ops.conv1x1(x, ws, cout, bias, sc), 20)
    t_t = timeit(lambda: F.conv2d(x, w, bias).mul_(sc), 20)
    nbytes = 4.0 * nb * (cin + cout) * H4 * W4
    print(f"conv1x1 {nb}x{cin}->{cout}: sa_conv1x1 {t_h:.1f} us ({nbytes / t_h / 1e3:.0f} GB/s), "
          f"F.conv2d {t_t:.1f} us")
mde = torch.rand(B, 1, 4 * H4, 4 * W4, device=dev)
outs = [torch.empty(B, 1, 4 * H4 >> i, 4 * W4 >> i, device=dev) for i in range(2, 6)]
t_h = timeit(lambda: ops.resample_multi(*[("interp", mde, o, None, None) for o in outs]), 20)
t_t = timeit(lambda: [F.interpolate(mde, scale_factor=1 / 2 ** i, mode="bilinear", align_corners=True)
                      for i in range(2, 6)], 20)
print(f"guidance pyramid (one image, 4 levels): resample_multi {t_h:.1f} us, F.interpolate {t_t:.1f} us")
