#!/usr/bin/env python3
"""The implicit-GEMM 3x3 conv (conv2d_igemm.hip, split f16 products on 16x16x32 MFMA) against the
F(4x4) split Winograd kernel on the model's conv shapes: max |error| vs torch fp32 (MIOpen) and the
kernel time (HIP events around `reps` back-to-back launches).
usage: python scripts/bench_igemm.py [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import _native as N, ops  # noqa: E402

SHAPES = [  # (B, Cin, Cout, H, W, tag)
    (4, 384, 256, 136, 240, "zr08"),
    (4, 256, 128, 136, 240, "qx08"),
    (4, 128, 256, 136, 240, "fh1"),
    (4, 128, 128, 136, 240, "qh08"),
    (4, 384, 256, 68, 120, "zr16"),
    (8, 128, 128, 136, 240, "fnet3"),
    (4, 256, 256, 34, 60, "zr32"),
]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    only = [a.split("=", 1)[1] for a in sys.argv[2:] if a.startswith("--only=")]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    print(f"{'conv':>6} {'shape':>24} {'igemm us':>9} {'wino4 us':>9} {'speedup':>7} {'ig TF/s':>8} "
          f"{'err ig':>9} {'err w4':>9}")
    for B, Cin, Cout, H, W, tag in SHAPES:
        if only and tag not in only:
            continue
        x = torch.randn(B, Cin, H, W, device=dev)
        w = torch.randn(Cout, Cin, 3, 3, device=dev) * (2.0 / (9 * Cin)) ** 0.5
        b = torch.randn(Cout, device=dev) * 0.1
        ref = torch.nn.functional.conv2d(x, w, b, padding=1)
        n = int(N.lib().sa_conv2d_igemm_weights_size(Cout, Cin))
        wig = torch.empty((n,), device=dev, dtype=torch.int32)
        N.call("sa_conv2d_igemm_weights", w.data_ptr(), Cout, Cin, wig.data_ptr(), 0)
        out = torch.empty_like(ref)
        prob = N.SaWinoProblem(x.data_ptr(), Cin * H * W, B, Cin, H, W, wig.data_ptr(), Cout, b.data_ptr(), 0,
                               None, None, None, 0, 0, out.data_ptr(), Cout * H * W, None, 0)
        gates = N.SaGateEpilogue()

        def ig():
            N.call("sa_conv2d_k3_igemm", 1, ctypes.addressof(prob), ctypes.addressof(gates), 0, 0)
        U = ops.wino_weights(w)

        def w4():
            ig_on, ops.IGEMM = ops.IGEMM, False   # the F(4x4) kernel, not the routed igemm
            try:
                return ops.conv2d_k3(x, U, bias=b)
            finally:
                ops.IGEMM = ig_on
        t_ig = timed(ig, reps)
        t_w4 = timed(w4, reps)
        if "--power" in sys.argv:
            # sysfs clock and board power while each kernel runs back to back for ~2 s
            import bench
            d = bench._gpu_sysfs(dev)
            for name, fn, t in (("igemm", ig, t_ig), ("wino4", w4, t_w4)):
                n_rep = max(1, int(2e6 / t))
                with bench.BoxSampler(d, 0.05) as smp:
                    for _ in range(n_rep):
                        fn()
                    torch.cuda.synchronize()
                print(f"   {name}: {smp.summary()}", flush=True)
        ig()
        o4 = w4()
        torch.cuda.synchronize()
        scale = ref.abs().max().item()
        e_ig = (out - ref).abs().max().item() / scale
        e_w4 = (o4 - ref).abs().max().item() / scale
        flops = 2.0 * B * Cin * Cout * 9 * H * W
        print(f"{tag:>6} {f'{B}x{Cin}->{Cout}@{H}x{W}':>24} {t_ig:9.1f} {t_w4:9.1f} {t_w4 / t_ig:7.2f} "
              f"{flops / t_ig / 1e6:8.1f} {e_ig:9.2e} {e_w4:9.2e}", flush=True)


if __name__ == "__main__":
    main()
