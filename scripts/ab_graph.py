#!/usr/bin/env python3
"""Forward at the bench config (B=4 pairs 544x960, 22 iterations) eager vs replayed from a
hipGraph captured with torch.cuda.graph (static input buffers refilled each step), for
ScheduleOptions.loop_parts / loop_offset combinations.
usage: python scripts/ab_graph.py [steps] [parts{T|F} ...]  (default 1T 2T 2F 3T 4T 4F)"""
import dataclasses
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, out


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    model = StereoAnywhere(dict(bench.PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    inp = bench.make_inputs(4, 540, 960, 544, 960, 192.0, seed0=1, device=dev)
    x = [inp["left"], inp["right"], inp["mono_left"], inp["mono_right"]]
    static = [t.clone() for t in x]
    base = model.opts
    ref = None
    with torch.no_grad():
        combos = [(int(a[:-1]), a[-1] == "T") for a in sys.argv[2:]] or \
            [(1, True), (2, True), (2, False), (3, True), (4, True), (4, False)]
        for parts, offset in combos:
            model.opts = dataclasses.replace(base, loop_parts=parts, loop_offset=offset)
            t_e, out_e = timed(lambda: model(*x, iters=22, test_mode=True)[0], 1 if parts > 1 else steps)
            if ref is None:
                ref = out_e
            # capture (after the eager warm-up: derived weights and MIOpen plans exist)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                model(*static, iters=22, test_mode=True)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                gout = model(*static, iters=22, test_mode=True)[0]

            def replay():
                for d, t in zip(static, x):
                    d.copy_(t)
                g.replay()
                return gout
            t_g, out_g = timed(replay, steps)
            print(f"loop_parts {parts} offset {offset}: eager {t_e:.2f} ms/step, graph {t_g:.2f} ms/step; "
                  f"max|d| eager {float((out_e - ref).abs().max()):.1e} graph {float((out_g - ref).abs().max()):.1e}",
                  flush=True)


if __name__ == "__main__":
    main()
