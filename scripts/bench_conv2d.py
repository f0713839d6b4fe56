#!/usr/bin/env python3
"""Fused Winograd conv (ops.conv2d_k3) vs torch/MIOpen fp32 conv at the model's 3x3 shapes
(B = 4 pairs at 544x960): per-call time with HIP events, and the max deviation."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402

SHAPES = [  # (name, N, Cin, Cout, H, W)
    ("fnet.layer1", 8, 64, 64, 544, 960), ("fnet.layer2", 8, 96, 96, 272, 480),
    ("fnet.layer3", 8, 128, 128, 136, 240), ("xc08", 4, 256, 384, 136, 240), ("hzr08", 4, 128, 256, 136, 240),
    ("qh08", 4, 128, 128, 136, 240), ("mot", 4, 192, 128, 136, 240), ("convc2", 8, 64, 64, 136, 240),
    ("xc16", 4, 256, 384, 68, 120), ("hzr16", 4, 128, 256, 68, 120), ("xc32", 4, 128, 384, 34, 60),
]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


def main():
    torch.backends.cudnn.benchmark = "--find" in sys.argv
    dev = torch.device("cuda", 0)
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--shape=")]
    for name, N, Cin, Cout, H, W in SHAPES:
        if only and name not in only:
            continue
        x = torch.randn(N, Cin, H, W, device=dev)
        w = torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)
        U = ops.wino_weights(w)
        out = torch.empty(N, Cout, H, W, device=dev)
        ops._WINO4 = False
        t_w = timeit(lambda: ops.conv2d_k3(x, U, out=out))
        ops._WINO4 = True
        t_4 = timeit(lambda: ops.conv2d_k3(x, U, out=out))
        f4 = float((ops.conv2d_k3(x, U) - F.conv2d(x, w, None, padding=1)).abs().max())
        if "--split" in sys.argv:   # F(4x4) fp32 MFMA vs the split kernel (block_shape 6)
            ops.W4_SPLIT = True
            Us = ops.wino_weights(w)
            t_s = timeit(lambda: ops.conv2d_k3(x, Us, out=out))
            fs = float((ops.conv2d_k3(x, Us) - F.conv2d(x, w, None, padding=1)).abs().max())
            ops.W4_SPLIT = False
            ex = 2.0 * 36 * N * Cout * Cin * ((H + 3) // 4) * ((W + 3) // 4)
            print(f"{name:12s} wino4 {t_4:8.1f} us ({ex / t_4 / 1e6:6.1f} TF exec) max|d| {f4:.2e}   "
                  f"split {t_s:8.1f} us ({ex / t_s / 1e6:6.1f} TF exec) max|d| {fs:.2e}  x{t_4 / t_s:.2f}", flush=True)
            continue
        if "--only-wino" in sys.argv:
            fl = 2.0 * N * Cout * Cin * 9 * H * W
            print(f"{name:12s} wino {t_w:8.1f} us ({fl / t_w / 1e6:6.1f} TF-eq)  wino4 {t_4:8.1f} us "
                  f"({fl / t_4 / 1e6:6.1f} TF-eq, {fl / 4 / t_4 / 1e6:5.1f} TF executed) max|d| {f4:.2e}", flush=True)
            continue
        t_m = timeit(lambda: F.conv2d(x, w, None, padding=1))
        ref = F.conv2d(x, w, None, padding=1)
        err = float((out - ref).abs().max())
        flops = 2.0 * N * Cout * Cin * 9 * H * W
        print(f"{name:12s} N{N} {Cin:4d}->{Cout:4d} {H}x{W}: wino {t_w:8.1f} us ({flops / t_w / 1e6:6.1f} TF-eq)"
              f"  miopen {t_m:8.1f} us ({flops / t_m / 1e6:6.1f})  max|d| {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
