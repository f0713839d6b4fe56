#!/usr/bin/env python3
"""Evaluation CLI with the reference test.py interface (test.py:34-103, run 161-249,
main 276-403), running the MI355X build.

Same flags, same per-sample procedure:
  iscale / oscale nearest resampling (test.py:169-176) -> mono maps (precomputed files,
  zeros for --monomodel none, or the synthetic set's own) -> replicate pad to ×32 (left/top
  get pad//2, 206-213) -> forward(test_mode=True) -> negate -> unpad -> rescale (238-240)
  -> guided_metrics (losses.py:273-342); a ground truth without points gives the metrics of
  an all-zero prediction (182-187); --stereomodel skip_pred predicts zeros (219-228).
Over --tries: per-try sample means, then mean / std over tries, printed as the reference's
MEAN / STD tables and written with its write_csv_header / write_csv_row (251-274, 347-403).
--monomodel DAv2 runs the Depth Anything V2 producer (stereoanywhere_amd/mono.py) when
--loadmonomodel names a checkpoint (or `seeded`), on both views stacked, min-max normalised
jointly (test.py:189-199); without --loadmonomodel the precomputed maps (--mono_tag) are read.  Datasets: `middlebury` (folder layout of
middlebury_dataset.py) and `synthetic` (seeded pairs with true disparity).
The tiled harness (configs 3 and 5) is test_mapreduce_v2.py.
Multi-GPU: run under torchrun; samples are split across ranks and the per-sample metric
rows are all-gathered to rank 0 (the only exchange).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from stereoanywhere_amd import data, dist, harness, metrics, mono, synth, tiler  # noqa: E402
from stereoanywhere_amd.checkpoint import load_reference_checkpoint  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

def build_parser():
    p = argparse.ArgumentParser(description="StereoAnywhere (MI355X build)")
    p.add_argument("--maxdisp", type=int, default=192)
    p.add_argument("--stereomodel", default="stereoanywhere")
    p.add_argument("--datapath", default="dataset/oak_dataset/")
    p.add_argument("--dataset", default="middlebury")
    p.add_argument("--outdir", default=None)
    p.add_argument("--loadstereomodel", default=None, help="reference .tar checkpoint (omit: seeded weights)")
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--iscale", type=float, default=1.0)
    p.add_argument("--oscale", type=float, default=1.0)
    p.add_argument("--tries", type=int, default=1)
    p.add_argument("--csv_path", default=None)
    p.add_argument("--mixed_precision", action="store_true")
    p.add_argument("--numworkers", type=int, default=1)
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--errormetric", default="bad 3.0", choices=["bad 1.0", "bad 2.0", "bad 3.0", "bad 4.0", "avgerr", "rms"])
    p.add_argument("--dilation", type=int, default=1)
    p.add_argument("--normalize", action="store_true")
    p.add_argument("--valsize", default=0, type=int)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--vanilla", action="store_true")
    p.add_argument("--monomodel", default="DAv2")
    p.add_argument("--loadmonomodel", default=None)
    p.add_argument("--preload_mono", action="store_true")
    p.add_argument("--vit_encoder", default="vitl", choices=["vitl", "vitb", "vits"])
    p.add_argument("--overfit", action="store_true", default=False)
    p.add_argument("--n_downsample", type=int, default=2)
    p.add_argument("--n_additional_hourglass", type=int, default=0)
    p.add_argument("--volume_channels", type=int, default=8)
    p.add_argument("--vol_downsample", type=float, default=0)
    p.add_argument("--vol_n_masks", type=int, default=8)
    p.add_argument("--use_truncate_vol", action="store_true")
    p.add_argument("--mirror_conf_th", type=float, default=0.98)
    p.add_argument("--mirror_attenuation", type=float, default=0.9)
    p.add_argument("--use_aggregate_stereo_vol", action="store_true")
    p.add_argument("--use_aggregate_mono_vol", action="store_true")
    p.add_argument("--normal_gain", type=int, default=10)
    p.add_argument("--lrc_th", type=float, default=1.0)
    p.add_argument("--iters", type=int, default=32)
    # build-specific
    p.add_argument("--mono_tag", default="dav2", help="file tag of precomputed mono maps (im0_<tag>.png)")
    p.add_argument("--synthetic_size", default="540x960", help="HxW of --dataset synthetic")
    p.add_argument("--synthetic_count", type=int, default=4)
    return p


def build_dataset(args):
    if args.dataset == "synthetic":
        h, w = map(int, args.synthetic_size.split("x"))
        return data.SyntheticPairs(args.synthetic_count, h, w, float(args.maxdisp))
    return data.dataset_for(args.dataset, args.datapath, None if args.monomodel == "none" else args.mono_tag)


@torch.no_grad()
def run(net, sample, args, device, mono_model=None):
    """test.py:161-249 for one sample (batch 1)."""
    t = {k: torch.from_numpy(np.ascontiguousarray(v))[None] for k, v in sample.items() if isinstance(v, np.ndarray)}
    t.setdefault("maskocc", torch.zeros_like(t["gt"]))
    if args.iscale != 1:
        t["im2"] = F.interpolate(t["im2"], scale_factor=1.0 / args.iscale)
        t["im3"] = F.interpolate(t["im3"], scale_factor=1.0 / args.iscale)
    if args.oscale != 1:
        t["gt"] = F.interpolate(t["gt"], scale_factor=1.0 / args.oscale, mode="nearest") / args.oscale
        t["validgt"] = F.interpolate(t["validgt"].float(), scale_factor=1.0 / args.oscale, mode="nearest")
        t["maskocc"] = F.interpolate(t["maskocc"].float(), scale_factor=1.0 / args.oscale, mode="nearest")
    if t["gt"].max() == 0:
        # test.py:182-187: no ground-truth point -> metrics of an all-zero prediction
        res = metrics.guided_metrics(torch.zeros_like(t["gt"]).numpy(), t["gt"].numpy(), t["validgt"].numpy(),
                                     t["maskocc"].numpy())
        res["disp"] = torch.ones_like(t["gt"]).squeeze(1)
        return res
    im2, im3 = t["im2"].to(device), t["im3"].to(device)
    if mono_model is not None:
        m2, m3 = mono.mono_pair_test(mono_model, im2, im3, args.dataset)
    elif "im2_mono" in t and args.monomodel != "none":
        m2, m3 = t["im2_mono"].to(device), t["im3_mono"].to(device)
        if m2.shape[-2:] != im2.shape[-2:]:
            m2 = F.interpolate(m2, size=im2.shape[-2:], mode="bilinear", align_corners=False)
            m3 = F.interpolate(m3, size=im3.shape[-2:], mode="bilinear", align_corners=False)
        lo, hi = torch.minimum(m2.min(), m3.min()), torch.maximum(m2.max(), m3.max())
        m2, m3 = (m2 - lo) / (hi - lo), (m3 - lo) / (hi - lo)  # joint min-max (test.py:198)
    else:
        m2, m3 = torch.zeros_like(im2[:, :1]), torch.zeros_like(im3[:, :1])
    pad = tiler.pad32(*im2.shape[-2:])

    def P(x):
        return F.pad(x, pad, mode="replicate")
    if args.stereomodel == "skip_pred":   # test.py:219-220, 227-228: zero prediction, no network
        pred = torch.zeros_like(P(im2))[:, 0]
    else:
        flow_up, _ = net(P(im2), P(im3), P(m2), P(m3), test_mode=True, iters=args.iters)
        pred = -flow_up[:, 0]
    hd, wd = pred.shape[-2:]
    pred = pred[..., pad[2]:hd - pad[3], pad[0]:wd - pad[1]]
    if args.iscale != 1 and args.iscale / args.oscale != 1:
        pred = F.interpolate(pred[None], t["gt"].shape[-2:], mode="nearest")[0] * args.iscale / args.oscale
    res = metrics.guided_metrics(pred.cpu().numpy(), t["gt"][:, 0].numpy(), t["validgt"][:, 0].numpy(),
                                 t["maskocc"][:, 0].numpy())
    res["disp"] = pred
    return res


def main(argv=None):
    """test.py:276-403: every try walks the (sharded) samples; metrics are aggregated over
    samples per try, then over tries (harness.aggregate_tries); CSV as write_csv_row."""
    args = build_parser().parse_args(argv)
    assert args.iscale > 0 and args.oscale > 0
    if args.no_cuda or not torch.cuda.is_available():
        raise SystemExit("the MI355X build runs on the GPU only (no CPU path)")
    if args.stereomodel not in ("stereoanywhere", "skip_pred"):
        raise SystemExit("no model")
    torch.manual_seed(args.seed)
    r = dist.init_from_env("nccl")
    device = torch.device("cuda", r.local_rank)
    net = None
    if args.stereomodel == "stereoanywhere":
        net = StereoAnywhere(vars(args)).eval()
        if args.loadstereomodel:
            load_reference_checkpoint(net, args.loadstereomodel)
        else:
            synth.load_seeded_weights(net, 0)
        net = net.to(device)
    mono_model = mono.load_for_harness(args, device)
    ds = build_dataset(args)
    n = len(ds) if args.valsize <= 0 else min(args.valsize, len(ds))

    def on_result(attempt, i, res):
        if args.outdir and attempt == 0:
            os.makedirs(args.outdir, exist_ok=True)
            data.write_pfm(os.path.join(args.outdir, f"{ds[i]['name']}_disp.pfm"), res["disp"][0].cpu().numpy())
        if args.verbose:
            print(f"{i}) " + ", ".join(f"{k}: {float(res[k])}" for k in harness.METRIC_ORDER))
    out = harness.evaluate(lambda i: run(net, ds[i], args, device, mono_model), n, args.tries, r, device, on_result)
    if out is None:
        return None
    acc_mean, acc_std = out
    print("\n".join(harness.summary_lines(acc_mean, acc_std)))
    if args.csv_path is not None:
        harness.append_csv(args.csv_path, args, acc_mean)
    return acc_mean


if __name__ == "__main__":
    main()
