#!/usr/bin/env python3
"""Direct fp32-MFMA conv (ops.conv_direct) vs torch/MIOpen at the encoder shapes of the bench
(fnet on 8 images, cnet on 4, 544x960): per-call time with HIP events."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import ops  # noqa: E402

SHAPES = [  # (name, N, Cin, Cout, H, W, K, S)
    ("fnet.stem", 8, 3, 64, 544, 960, 7, 1), ("cnet.stem", 4, 3, 64, 544, 960, 7, 1),
    ("fnet.l2", 8, 64, 96, 544, 960, 3, 2), ("fnet.l3", 8, 96, 128, 272, 480, 3, 2),
    ("cnet.l4", 4, 128, 128, 136, 240, 3, 2),
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
    dev = torch.device("cuda", 0)
    for name, N, Cin, Cout, H, W, K, S in SHAPES:
        x = torch.randn(N, Cin, H, W, device=dev)
        w = torch.randn(Cout, Cin, K, K, device=dev) / (K * Cin ** 0.5)
        wg = ops.conv_direct_weights(w, S)
        wd = None
        if S == 2:
            wdr = torch.randn(Cout, Cin, 1, 1, device=dev) / Cin ** 0.5
            wd = ops.conv_direct_weights(wdr, S, with_ds=True)
        t = timeit(lambda: ops.conv_direct(x, wg, K, S, Cout, wd=wd))
        if "--split" in sys.argv:   # fp32 products vs the split kernel (ops.DIRECT_SPLIT)
            res = {}
            for sp in (False, True):
                ops.DIRECT_SPLIT = sp
                g_ = ops.conv_direct_weights(w, S)
                d_ = ops.conv_direct_weights(wdr, S, with_ds=True) if S == 2 else None
                res[sp] = timeit(lambda: ops.conv_direct(x, g_, K, S, Cout, wd=d_))
            print(f"{name:10s} fp32 {res[False]:8.1f} us   split {res[True]:8.1f} us  x{res[False] / res[True]:.2f}",
                  flush=True)
            continue
        Ho, Wo = (H + 2 * (K // 2) - K) // S + 1, (W + 2 * (K // 2) - K) // S + 1
        fl = 2.0 * N * Cout * Cin * K * K * Ho * Wo + (2.0 * N * Cout * Cin * Ho * Wo if wd is not None else 0)
        tm = timeit(lambda: F.conv2d(x, w, None, S, K // 2))
        if wd is not None:
            tm += timeit(lambda: F.conv2d(x, wdr, None, S, 0))
        print(f"{name:10s} direct {t:8.1f} us ({fl / t / 1e6:6.1f} TF)   miopen {tm:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
