#!/usr/bin/env python3
"""Eager forward vs hipGraph replay of the same forward (bench workload: 4 pairs at 544x960,
22 iterations): time per step, and the max difference of the outputs."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

PUBLISHED = dict(use_truncate_vol=True, use_aggregate_mono_vol=True, vol_n_masks=8, n_additional_hourglass=0,
                 vol_downsample=0, mirror_conf_th=0.98, mirror_attenuation=0.9, lrc_th=1.0, normal_gain=10)


def main():
    dev = torch.device("cuda", 0)
    m = StereoAnywhere(dict(PUBLISHED)).eval()
    synth.load_seeded_weights(m, 0)
    m = m.to(dev)
    p = synth.synthetic_batch(4, 544, 960, 192.0, seed0=1)
    x = [torch.from_numpy(p[k]).to(dev) for k in ("left", "right", "mono_left", "mono_right")]
    with torch.no_grad():
        for _ in range(2):
            ref = m(*x, iters=22, test_mode=True)[0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            m(*x, iters=22, test_mode=True)
        torch.cuda.synchronize()
        print(f"eager {1e3 * (time.perf_counter() - t0) / 5:.2f} ms/step", flush=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(*x, iters=22, test_mode=True)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = m(*x, iters=22, test_mode=True)[0]
        g.replay()
        torch.cuda.synchronize()
        print("graph max diff vs eager", float((out - ref).abs().max()), flush=True)
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        print(f"graph {1e3 * (time.perf_counter() - t0) / 5:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
