#!/usr/bin/env python3
"""Same-box A/B of the bench forward (4 pairs at 544x960, 22 iterations) under environment
settings given as NAME=VALUE,... groups; each setting runs in a fresh child process, the
list is interleaved twice."""
import os
import subprocess
import sys

CHILD = r"""
import os, sys, time, torch
sys.path.insert(0, os.environ["SA_ROOT"])
from stereoanywhere_amd import synth
from stereoanywhere_amd.model import StereoAnywhere
from stereoanywhere_amd import ops
ops.W4_QUAD = os.environ.get("SA_AB_W4_QUAD") == "1"
P = dict(use_truncate_vol=True, use_aggregate_mono_vol=True, vol_n_masks=8, n_additional_hourglass=0,
         vol_downsample=0, mirror_conf_th=0.98, mirror_attenuation=0.9, lrc_th=1.0, normal_gain=10)
m = StereoAnywhere(dict(P)).eval(); synth.load_seeded_weights(m, 0); m = m.cuda()
p = synth.synthetic_batch(4, 544, 960, 192.0, seed0=1)
x = [torch.from_numpy(p[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
with torch.no_grad():
    for _ in range(2): m(*x, iters=22, test_mode=True)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(5): m(*x, iters=22, test_mode=True)
    torch.cuda.synchronize()
print(f"{1e3 * (time.perf_counter() - t) / 5:.2f}")
"""


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    settings = sys.argv[1:] or [""]
    for rnd in range(2):
        for st in settings:
            env = dict(os.environ, SA_ROOT=root)
            for kv in filter(None, st.split(",")):
                k, v = kv.split("=", 1)
                env[k] = v
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(st, "FAILED", r.stderr[-2000:])
                sys.exit(1)
            print(f"round {rnd} [{st or 'default'}] {r.stdout.strip()} ms/step", flush=True)


if __name__ == "__main__":
    main()
