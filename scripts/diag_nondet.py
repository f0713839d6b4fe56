#!/usr/bin/env python3
"""Run-to-run determinism of the forward at cfg2 (batch 4, 540x960, 22 iterations): the same eager
forward three times per setting, max |difference| of the disparity between runs, for the kernel
switches given as name=value pairs of ops module flags (e.g. W4_SPLIT=0 CONV3D_MFMA=1) and the
model's stream overlap (overlap=0/1).
usage: python scripts/diag_nondet.py [iters] [FLAG=v ...] [overlap=0|1]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import PUBLISHED, make_inputs  # noqa: E402
from stereoanywhere_amd import ops, synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 22
    overlap = True
    for a in sys.argv[1:]:
        if "=" in a:
            k, v = a.split("=")
            if k == "overlap":
                overlap = v == "1"
            else:
                setattr(ops, k, bool(int(v)))
                print(f"ops.{k} = {getattr(ops, k)}")
    dev = torch.device("cuda", 0)
    model = StereoAnywhere(dict(PUBLISHED)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    model.stream_overlap = overlap
    inp = make_inputs(4, 540, 960, 544, 960, 192.0, seed0=1, device=dev)
    x = (inp["left"], inp["right"], inp["mono_left"], inp["mono_right"])
    outs = []
    with torch.no_grad():
        for _ in range(3):
            flow, _ = model(*x, iters=iters, test_mode=True)
            torch.cuda.synchronize()
            outs.append(flow.clone())
    d01 = float((outs[0] - outs[1]).abs().max())
    d02 = float((outs[0] - outs[2]).abs().max())
    d12 = float((outs[1] - outs[2]).abs().max())
    print(f"{' '.join(a for a in sys.argv[1:] if '=' in a)} iters={iters}: "
          f"run-to-run max |d| 0-1 {d01:.3g} 0-2 {d02:.3g} 1-2 {d12:.3g}", flush=True)


if __name__ == "__main__":
    main()
