#!/usr/bin/env python3
"""Forward time at the bench config (B=4 pairs 544x960, 22 iterations, side streams on) for
ScheduleOptions.loop_parts = 1, 2, 4 (the GRU loop's batch parts on separate streams).
usage: python scripts/ab_loop_parts.py [steps]"""
import dataclasses
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    model = StereoAnywhere(dict(bench.PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    inp = bench.make_inputs(4, 540, 960, 544, 960, 192.0, seed0=1, device=dev)
    x = (inp["left"], inp["right"], inp["mono_left"], inp["mono_right"])
    base = model.opts
    outs = {}
    with torch.no_grad():
        for rnd in range(2):
            for parts in (1, 2, 4):
                model.opts = dataclasses.replace(base, loop_parts=parts)
                model(*x, iters=22, test_mode=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    out = model(*x, iters=22, test_mode=True)[0]
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / steps * 1e3
                outs.setdefault(parts, out)
                d = float((out - outs[1]).abs().max())
                print(f"round {rnd} loop_parts {parts}: {dt:.2f} ms/step ({4e3 / dt:.2f} pairs/s) max|d| vs 1: {d:.2e}",
                      flush=True)


if __name__ == "__main__":
    main()
