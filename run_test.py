#!/usr/bin/env python3
"""Launcher with the reference run_test.py flag set (run_test.py:53-81), paths from the
command line instead of hard-coded ones.  Runs test.py in a child process (one GPU) or
under torchrun with --gpus N (one process per GPU)."""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))

# published evaluation flags (README.md:314-321; run_test.py:62-74)
PUBLISHED = ["--stereomodel", "stereoanywhere", "--iters", "32", "--vol_n_masks", "8", "--n_additional_hourglass",
             "0", "--use_aggregate_mono_vol", "--vol_downsample", "0", "--mirror_conf_th", "0.98",
             "--use_truncate_vol", "--mirror_attenuation", "0.9", "--normalize", "--preload_mono"]


def command(args, extra):
    cmd = [sys.executable]
    if args.gpus > 1:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
                "--master-addr", "127.0.0.1", f"--master-port={args.port}"]
    cmd += [os.path.join(ROOT, "test.py"), "--datapath", args.datapath, "--dataset", args.dataset,
            "--monomodel", args.monomodel, "--iscale", str(args.iscale), "--oscale", str(args.oscale)] + PUBLISHED
    if args.loadstereomodel:
        cmd += ["--loadstereomodel", args.loadstereomodel]
    return cmd + extra


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--datapath", default="datasets/mb2014/trainingH")
    ap.add_argument("--dataset", default="middlebury")
    ap.add_argument("--loadstereomodel", default=None)
    ap.add_argument("--monomodel", default="DAv2")
    ap.add_argument("--iscale", type=float, default=1.0)
    ap.add_argument("--oscale", type=float, default=1.0)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--port", type=int, default=29511)
    args, extra = ap.parse_known_args()
    cmd = command(args, extra)
    print("running:", " ".join(cmd))
    sys.exit(subprocess.run(cmd).returncode)


if __name__ == "__main__":
    main()
