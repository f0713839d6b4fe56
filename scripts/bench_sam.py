#!/usr/bin/env python3
"""soft-argmin + confidence (sa_softargmin_conf) at the model's layout and size: two volumes
as channel views of one [4, 2, 240, 136, 240] tensor ([B, 2, W2, H, W1]), HIP events per call.
SA_HIP_LIB selects the library (A/B against a variant build)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv2d import timeit  # noqa: E402

B, H, W = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (4, 136, 240)))
t = torch.randn(B, 2, W, H, W, device="cuda") * 4
vd, vc = t[:, 0:1], t[:, 1:2]
strides = (t.stride(0), W, 1, H * W)
alg = 2 * 4 * B * H * W * W
from stereoanywhere_amd import _native as N  # noqa: E402
NAMES = {1: "one-pass", 2: "one-pass (16-byte rows where they apply)", 0: "per-line"}
for one_pass in (1, 2, 0):
    N.lib().sa_softargmin_set_one_pass(one_pass)
    us = timeit(lambda: ops.softargmin_conf(vd, vc, strides, (B, H, W, W)), reps=20)
    print(f"softargmin_conf {B}x{H}x{W}x{W} {NAMES[one_pass]}: {us:.1f} us, "
          f"{alg / us / 1e6:.2f} TB/s of algorithmic bytes ({alg / 1e6:.0f} MB)", flush=True)
N.lib().sa_softargmin_set_one_pass(1)
