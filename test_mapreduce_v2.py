#!/usr/bin/env python3
"""Tiled evaluation CLI with the reference test_mapreduce_v2.py interface (flags 32-87,
run_mapreduce 178-301, main 363-592), running the MI355X build through the mapreduce_v2-
compatible tiler (stereoanywhere_amd/tiler.py).  Configs 3 and 5 (Middlebury-H, Booster).

Per sample, as the reference does:
  bilinear ``iscale`` down-sampling of the images (194), nearest ``oscale`` of the ground
  truth -> mono maps min-max normalised jointly over the stacked pair with +1e-8 (159;
  --monomodel DAv2 with --loadmonomodel <checkpoint | seeded> runs the Depth Anything V2
  producer, stereoanywhere_amd/mono.py, at compute_mono_pair's input size, 113-160; without
  --loadmonomodel the precomputed maps; zeros for --monomodel none) ->
  replicate pad to x32 (left/top get pad//2) -> uint8 truncation of the padded images
  (tensor_to_numpy_image, 163-175, 229-230) -> MapReduceInference.infer(iscale=1,
  oscale=1, iters, test_mode=True) -> unpad -> nearest resize to the ground truth
  (262-282) -> guided_metrics.
Tiling: --tile_preset (name / 'auto' by dataset / 'list'), else --tile_width/--tile_height
(rectangular) or --tile_size (square), --overlap, 0 = the VRAM heuristic.
Multi-GPU: run under torchrun; samples are split across ranks and the per-sample metric rows
are all-gathered to rank 0.
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
from stereoanywhere_amd.offload import CPUOffloadWrapper  # noqa: E402

def build_parser():
    p = argparse.ArgumentParser(description="StereoAnywhere MapReduce evaluation (MI355X build)")
    p.add_argument("--datapath", default="dataset/")
    p.add_argument("--dataset", default="middlebury")
    p.add_argument("--loadstereomodel", default=None, help="reference .tar checkpoint (omit: seeded weights)")
    p.add_argument("--loadmonomodel", default=None)
    p.add_argument("--stereomodel", default="stereoanywhere")
    p.add_argument("--monomodel", default="DAv2")
    p.add_argument("--vit_encoder", default="vitl", choices=["vitl", "vitb", "vits"])
    p.add_argument("--maxdisp", type=int, default=192)
    p.add_argument("--iscale", type=float, default=1.0)
    p.add_argument("--oscale", type=float, default=1.0)
    p.add_argument("--tries", type=int, default=1)
    p.add_argument("--valsize", type=int, default=0)
    p.add_argument("--mixed_precision", action="store_true")
    p.add_argument("--half", action="store_true")
    p.add_argument("--errormetric", default="bad 3.0")
    p.add_argument("--dilation", type=int, default=1)
    p.add_argument("--outdir", default=None)
    p.add_argument("--csv_path", default=None)
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--numworkers", type=int, default=1)
    p.add_argument("--normalize", action="store_true")
    p.add_argument("--iters", type=int, default=32)
    p.add_argument("--vol_n_masks", type=int, default=8)
    p.add_argument("--vol_downsample", type=float, default=0)
    p.add_argument("--use_truncate_vol", action="store_true")
    p.add_argument("--use_aggregate_mono_vol", action="store_true")
    p.add_argument("--use_aggregate_stereo_vol", action="store_true")
    p.add_argument("--mirror_conf_th", type=float, default=0.95)
    p.add_argument("--mirror_attenuation", type=float, default=0.85)
    p.add_argument("--overfit", action="store_true", default=False)
    p.add_argument("--tile_preset", type=str, default=None)
    p.add_argument("--tile_size", type=int, default=0)
    p.add_argument("--tile_width", type=int, default=0)
    p.add_argument("--tile_height", type=int, default=0)
    p.add_argument("--overlap", type=int, default=0)
    p.add_argument("--batch_tiles", action="store_true")
    p.add_argument("--clear_cache", action="store_true")
    p.add_argument("--non_lambertian", action="store_true")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--use_global_guidance", action="store_true")
    p.add_argument("--guidance_scale", type=float, default=2.0)
    p.add_argument("--guidance_weight", type=float, default=0.3)
    p.add_argument("--guidance_dir", type=str, default=None, help="[deprecated in the reference; ignored]")
    # build-specific
    p.add_argument("--mono_tag", default="dav2", help="file tag of precomputed mono maps (im0_<tag>.png)")
    p.add_argument("--synthetic_size", default="540x960", help="HxW of --dataset synthetic")
    p.add_argument("--synthetic_count", type=int, default=4)
    p.add_argument("--cpu_offload", action="store_true",
                   help="run the tiler under CPUOffloadWrapper (cpu_offload_wrapper.py:28-83; config 5)")
    return p


def build_dataset(args):
    if args.dataset == "synthetic":
        h, w = map(int, args.synthetic_size.split("x"))
        return data.SyntheticPairs(args.synthetic_count, h, w, float(args.maxdisp))
    return data.dataset_for(args.dataset, args.datapath, None if args.monomodel == "none" else args.mono_tag)


def apply_preset(args) -> bool:
    """main 367-389: a preset fills the tile sides / overlap not given explicitly.
    Returns False for --tile_preset list (prints the table)."""
    if not args.tile_preset:
        return True
    if args.tile_preset.lower() == "list":
        for p in tiler.TILE_PRESETS.values():
            print(f"[{p.name}] {p.tile_width}x{p.tile_height} overlap {p.overlap}")
        return False
    p = (tiler.get_preset_for_dataset(args.dataset) if args.tile_preset.lower() == "auto"
         else tiler.get_preset(args.tile_preset))
    if args.tile_width <= 0:
        args.tile_width = p.tile_width
    if args.tile_height <= 0:
        args.tile_height = p.tile_height
    if args.overlap <= 0:
        args.overlap = p.overlap
    return True


def build_inferencer(net, args, rank: int = 0, world: int = 1) -> tiler.MapReduceInference:
    """main 405-468: rectangular tiles when both sides are set, else square (0 = heuristic)."""
    if args.non_lambertian:
        raise NotImplementedError("NonLambertianProcessor is broken in the reference (SURVEY §4) and not built")
    common = dict(mono_model=None, batch_tiles=args.batch_tiles, mixed_precision=args.mixed_precision,
                  clear_cache=args.clear_cache, use_global_guidance=args.use_global_guidance,
                  guidance_scale=args.guidance_scale, guidance_weight=args.guidance_weight, rank=rank, world=world)
    if args.tile_width > 0 and args.tile_height > 0:
        ov = args.overlap if args.overlap > 0 else tiler.select_tiling_parameters().overlap
        return tiler.MapReduceInference(net, tile_width=args.tile_width, tile_height=args.tile_height, overlap=ov,
                                        **common)
    if args.tile_size <= 0 or args.overlap <= 0:
        p = tiler.select_tiling_parameters()
        ts, ov = p.tile_size, p.overlap
    else:
        ts, ov = args.tile_size, args.overlap
    return tiler.MapReduceInference(net, tile_size=ts, overlap=ov, **common)


@torch.no_grad()
def run_mapreduce(sample, args, device, inferencer: tiler.MapReduceInference, mono_model=None) -> dict:
    """test_mapreduce_v2.py:178-301 for one sample (batch 1)."""
    t = {k: torch.from_numpy(np.ascontiguousarray(v))[None] for k, v in sample.items() if isinstance(v, np.ndarray)}
    t.setdefault("maskocc", torch.zeros_like(t["gt"]))
    if args.iscale != 1:
        for k in ("im2", "im3"):
            t[k] = F.interpolate(t[k], scale_factor=1.0 / args.iscale, mode="bilinear", align_corners=False)
    if args.oscale != 1:
        t["gt"] = F.interpolate(t["gt"], scale_factor=1.0 / args.oscale, mode="nearest") / args.oscale
        t["validgt"] = F.interpolate(t["validgt"].float(), scale_factor=1.0 / args.oscale, mode="nearest")
        t["maskocc"] = F.interpolate(t["maskocc"].float(), scale_factor=1.0 / args.oscale, mode="nearest")
    im2, im3 = t["im2"].to(device), t["im3"].to(device)
    if mono_model is not None:
        m = mono.mono_pair_mapreduce(mono_model, im2, im3, args.dataset)
        ml, mr = m[0:1], m[1:2]
    elif "im2_mono" in t and args.monomodel != "none":
        m = torch.cat([t["im2_mono"], t["im3_mono"]]).to(device)
        if m.shape[-2:] != im2.shape[-2:]:
            m = F.interpolate(m, size=im2.shape[-2:], mode="bilinear", align_corners=False)
        m = (m - m.min()) / (m.max() - m.min() + 1e-8)   # joint over the stacked pair (159)
        ml, mr = m[0:1], m[1:2]
    else:
        ml, mr = torch.zeros_like(im2[:, :1]), torch.zeros_like(im3[:, :1])
    pad = tiler.pad32(*im2.shape[-2:])

    def P(x):
        return F.pad(x, pad, mode="replicate")
    im2p = P(im2)
    disp = inferencer.infer(tiler.to_uint8_image(im2p), tiler.to_uint8_image(P(im3)), iscale=1.0, oscale=1.0,
                            mono_size=tuple(im2p.shape[-2:]), verbose=args.verbose, mono_pair=(P(ml), P(mr)),
                            iters=args.iters, test_mode=True)
    d = torch.from_numpy(np.asarray(disp)).float()
    d = d[None, None] if d.dim() == 2 else d.unsqueeze(1) if d.dim() == 3 else d
    hd, wd = d.shape[-2:]
    d = d[..., pad[2]:hd - pad[3], pad[0]:wd - pad[1]]
    gt = t["gt"]
    if args.iscale != 1 and args.iscale / args.oscale != 1:
        d = F.interpolate(d, size=gt.shape[-2:], mode="nearest") * args.iscale / args.oscale
    elif d.shape[-2:] != gt.shape[-2:]:
        w0 = d.shape[-1]
        d = F.interpolate(d, size=gt.shape[-2:], mode="nearest") * (gt.shape[-1] / w0)
    res = metrics.guided_metrics(d[:, 0].numpy(), gt[:, 0].numpy(), t["validgt"][:, 0].numpy(),
                                 t["maskocc"][:, 0].numpy())
    res["disp"] = d[:, 0]
    return res


def main(argv=None):
    args = build_parser().parse_args(argv)
    if not apply_preset(args):
        return None
    assert args.iscale > 0 and args.oscale > 0
    if args.no_cuda or not torch.cuda.is_available():
        raise SystemExit("the MI355X build runs on the GPU only (no CPU path)")
    if args.half:
        raise SystemExit("--half: the build computes in fp32 only")
    torch.manual_seed(args.seed)
    r = dist.init_from_env("nccl")
    device = torch.device("cuda", r.local_rank)
    net = StereoAnywhere(vars(args)).eval()
    if args.loadstereomodel:
        load_reference_checkpoint(net, args.loadstereomodel)
    else:
        synth.load_seeded_weights(net, 0)
    net = net.to(device)
    inferencer = build_inferencer(net, args)
    if args.cpu_offload:
        # config 5: the tiler runs under the offload wrapper (HBM-resident on MI355X, offload.py)
        inferencer.tile_wrapper = CPUOffloadWrapper(inferencer.tile_wrapper)
    mono_model = mono.load_for_harness(args, device)
    ds = build_dataset(args)
    n = len(ds) if args.valsize <= 0 else min(args.valsize, len(ds))

    def on_result(attempt, i, res):
        if args.outdir and attempt == 0:
            os.makedirs(args.outdir, exist_ok=True)
            data.write_pfm(os.path.join(args.outdir, f"{ds[i]['name']}_disp.pfm"), res["disp"][0].cpu().numpy())
        if args.verbose:
            print(ds[i]["name"], {k: round(float(res[k]), 4) for k in harness.METRIC_ORDER[:10]})
    out = harness.evaluate(lambda i: run_mapreduce(ds[i], args, device, inferencer, mono_model), n, args.tries, r, device,
                           on_result)
    if out is None:
        return None
    # test_mapreduce_v2.py:531-588: same aggregation as test.py, tables in guided_metrics order
    acc_mean, acc_std = out
    print("\n".join(harness.summary_lines(acc_mean, acc_std, harness.METRIC_ORDER)))
    if args.csv_path is not None:
        # the reference accepts --csv_path here but writes nothing; the build writes test.py's row
        harness.append_csv(args.csv_path, args, acc_mean)
    return acc_mean


if __name__ == "__main__":
    main()
