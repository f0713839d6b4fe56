"""Time the Depth Anything V2 producer (stereoanywhere_amd/mono.py) the way the harnesses
call it: both views of a pair stacked through infer_image, seeded weights (no checkpoint
offline).  Default: vitl on a Middlebury-H-sized pair (1008 x 1488) at test.py's
'middlebury' input size (1036 x 1036 lower bound -> 1036 x 1526).
usage: python scripts/bench_mono.py [--encoder vitl] [--size 1008x1488] [--dataset middlebury]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereoanywhere_amd import mono, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--encoder", default="vitl")
    ap.add_argument("--size", default="1008x1488")
    ap.add_argument("--dataset", default="middlebury")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    H, W = map(int, a.size.split("x"))
    m = mono.DepthAnythingV2(**mono.MODEL_CONFIGS[a.encoder])
    synth.load_seeded_weights(m, 0)
    m = m.cuda().eval()
    g = torch.Generator().manual_seed(0)
    im2, im3 = (torch.rand(1, 3, H, W, generator=g).cuda() for _ in range(2))
    for _ in range(2):
        mono.mono_pair_test(m, im2, im3, a.dataset)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        mono.mono_pair_test(m, im2, im3, a.dataset)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    fh, fw = mono.resize_target(H, W, mono.INPUT_WIDTH[a.dataset], mono.INPUT_HEIGHT[a.dataset])
    print(json.dumps({"producer": f"DAv2-{a.encoder}", "pair": f"{H}x{W}", "network_input": f"2x{fh}x{fw}",
                      "tokens_per_view": (fh // 14) * (fw // 14), "ms_per_pair": dt * 1e3, "pairs_per_s": 1.0 / dt}))


if __name__ == "__main__":
    main()
