#!/usr/bin/env python3
"""Why bench.py's one-stream leg of config 5 runs ~2.8x slower than its instrumented leg:
per-step wall times of one-stream steps, instrumented steps and one-stream steps again, with
the caching allocator's counters (alloc retries = cudaFree of cached blocks + re-malloc)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from stereoanywhere_amd import _native as N, synth, tiler  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402
from stereoanywhere_amd.offload import CPUOffloadWrapper  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = StereoAnywhere(dict(use_truncate_vol=True, use_aggregate_mono_vol=True)).eval()
    synth.load_seeded_weights(model, 0)
    model = model.to(dev)
    H, W = 3008, 4128
    pb = synth.synthetic_batch(1, H, W, 512.0, seed0=1)
    x = [torch.from_numpy(pb[k]).to(dev) for k in ("left", "right", "mono_left", "mono_right")]
    run = CPUOffloadWrapper(tiler.from_preset(model, "booster", batch_tiles=True))

    def step(tag):
        torch.cuda.synchronize()
        s0 = torch.cuda.memory_stats(dev)
        t0 = time.perf_counter()
        with torch.no_grad():
            run(*x, iters=32, test_mode=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s1 = torch.cuda.memory_stats(dev)
        print(f"{tag:14s} {dt * 1e3:8.1f} ms  retries +{s1['num_alloc_retries'] - s0['num_alloc_retries']}  "
              f"device mallocs +{s1.get('num_device_alloc', 0) - s0.get('num_device_alloc', 0)}  "
              f"reserved {s1['reserved_bytes.all.current'] / 2**30:.1f} GiB  "
              f"peak {s1['allocated_bytes.all.peak'] / 2**30:.1f} GiB", flush=True)
    for i in range(2):
        step(f"default {i}")
    model.stream_overlap = False
    for i in range(3):
        step(f"one-stream {i}")
    N.timing_enable(True)
    for i in range(2):
        step(f"instrumented {i}")
    N.timing_enable(False)
    for i in range(2):
        step(f"one-stream {i}")
    model.stream_overlap = True
    step("default again")


if __name__ == "__main__":
    main()
