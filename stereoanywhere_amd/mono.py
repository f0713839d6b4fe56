"""Depth Anything V2 mono producer (the mde2 / mde3 maps configs 3 and 5 feed the stereo path).

The reference bundles the upstream DAv2 code (models/depth_anything_v2/): a DINOv2 ViT
(dinov2.py:45-357) whose four intermediate blocks feed a DPT head (dpt.py:38-165), and the
harness calls ``infer_image`` on both views stacked (test.py:189-199,
test_mapreduce_v2.py:113-160) before min-max normalising them jointly.  This module is the
same network under the same state-dict names (so a ``depth_anything_v2_vit*.pth`` loads with
``strict=True``), written for MI355X inference:

* attention runs through ``F.scaled_dot_product_attention`` (one fused kernel per layer on
  ROCm) instead of the reference's explicit q·kᵀ / softmax / ·v (attention.py:55-67, its
  path without xFormers); the projections and the MLP are plain GEMMs (hipBLASLt);
* ``no_grad`` inference only: no stochastic depth, dropout or masking paths.

The producer sits outside the cost-volume hot path (the upstream model
that writes the mono maps), so it uses library kernels.  Parity: tests/golden/dav2.npz holds
the reference ``DepthAnythingV2('vits').infer_image`` output for seeded weights
(tests/golden/make_golden.py ``dav2_cases``; cv2 is absent here, and on this path the
reference uses it only for the interpolation-method constants its Resize object stores, so
the script provides those constants).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# depth_anything_v2/__init__.py:27-32
MODEL_CONFIGS = {
    "vits": dict(encoder="vits", features=64, out_channels=[48, 96, 192, 384]),
    "vitb": dict(encoder="vitb", features=128, out_channels=[96, 192, 384, 768]),
    "vitl": dict(encoder="vitl", features=256, out_channels=[256, 512, 1024, 1024]),
    "vitg": dict(encoder="vitg", features=384, out_channels=[1536, 1536, 1536, 1536]),
}
# dinov2.py:362-420: (embed_dim, depth, heads); vitg uses the fused SwiGLU FFN
_VIT = {"vits": (384, 12, 6), "vitb": (768, 12, 12), "vitl": (1024, 24, 16), "vitg": (1536, 40, 24)}
# dpt.py:172-177
INTERMEDIATE_LAYERS = {"vits": [2, 5, 8, 11], "vitb": [2, 5, 8, 11], "vitl": [4, 11, 17, 23], "vitg": [9, 19, 29, 39]}
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ---------------------------------------------------------------------------------------------
# DINOv2 ViT (dinov2.py, dinov2_layers/*)


class _PatchEmbed(nn.Module):
    def __init__(self, patch: int, dim: int):
        super().__init__()
        self.proj = nn.Conv2d(3, dim, kernel_size=patch, stride=patch)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)   # [B, N, D] (patch_embed.py:72-88)


class _Attention(nn.Module):
    def __init__(self, dim: int, heads: int):
        super().__init__()
        self.num_heads = heads
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        B, N, C = x.shape
        q, k, v = self.qkv(x).reshape(B, N, 3, self.num_heads, C // self.num_heads).permute(2, 0, 3, 1, 4)
        # softmax(q kᵀ / sqrt(d)) v, attention.py:55-67
        y = F.scaled_dot_product_attention(q, k, v)
        return self.proj(y.transpose(1, 2).reshape(B, N, C))


class _Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))   # mlp.py:34-41 (exact GELU)


class _SwiGLU(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        hidden = (int(hidden * 2 / 3) + 7) // 8 * 8   # swiglu_ffn.py:56-57
        self.w12 = nn.Linear(dim, 2 * hidden)
        self.w3 = nn.Linear(hidden, dim)

    def forward(self, x):
        x1, x2 = self.w12(x).chunk(2, dim=-1)
        return self.w3(F.silu(x1) * x2)


class _LayerScale(nn.Module):
    def __init__(self, dim: int):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return x * self.gamma


class _Block(nn.Module):
    def __init__(self, dim: int, heads: int, swiglu: bool):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _Attention(dim, heads)
        self.ls1 = _LayerScale(dim)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = (_SwiGLU if swiglu else _Mlp)(dim, 4 * dim)
        self.ls2 = _LayerScale(dim)

    def forward(self, x):   # block.py:103-120, eval branch
        x = x + self.ls1(self.attn(self.norm1(x)))
        return x + self.ls2(self.mlp(self.norm2(x)))


class DINOv2(nn.Module):
    """DinoVisionTransformer as DINOv2(model_name) builds it (dinov2.py:409-422): img_size 518,
    patch 14, LayerScale 1.0, no register tokens, no block chunks, interpolate offset 0.1."""

    def __init__(self, model_name: str = "vitl"):
        super().__init__()
        dim, depth, heads = _VIT[model_name]
        self.embed_dim, self.patch_size, self.interpolate_offset = dim, 14, 0.1
        n = (518 // 14) ** 2
        self.patch_embed = _PatchEmbed(14, dim)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, dim))
        self.blocks = nn.ModuleList([_Block(dim, heads, model_name == "vitg") for _ in range(depth)])
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.mask_token = nn.Parameter(torch.zeros(1, dim))   # unused at inference, kept for the state dict

    def _pos_embed(self, npatch: int, H: int, W: int) -> torch.Tensor:
        # dinov2.py:188-213: bicubic resize of the 37 x 37 grid by ((H/14 + 0.1)/37, (W/14 + 0.1)/37)
        N = self.pos_embed.shape[1] - 1
        if npatch == N and H == W:
            return self.pos_embed
        pos = self.pos_embed.float()
        side = math.sqrt(N)
        h0, w0 = H // self.patch_size + self.interpolate_offset, W // self.patch_size + self.interpolate_offset
        grid = pos[:, 1:].reshape(1, int(side), int(side), -1).permute(0, 3, 1, 2)
        grid = F.interpolate(grid, scale_factor=(float(h0) / side, float(w0) / side), mode="bicubic", antialias=False)
        if grid.shape[-2] != int(h0) or grid.shape[-1] != int(w0):
            raise RuntimeError(f"position grid resized to {tuple(grid.shape[-2:])}, expected {(int(h0), int(w0))}")
        grid = grid.permute(0, 2, 3, 1).reshape(1, -1, grid.shape[1])
        return torch.cat((pos[:, :1], grid), dim=1).to(self.pos_embed.dtype)

    def get_intermediate_layers(self, x: torch.Tensor, n: Sequence[int], return_class_token: bool = True):
        """Normalised patch tokens (and class tokens) after the blocks in ``n`` (dinov2.py:310-345)."""
        _, _, H, W = x.shape
        if H % 14 or W % 14:
            raise ValueError(f"input {H}x{W} is not a multiple of the 14-pixel patch")
        t = self.patch_embed(x)
        t = torch.cat((self.cls_token.expand(t.shape[0], -1, -1), t), dim=1)
        t = t + self._pos_embed(t.shape[1] - 1, H, W)
        take, outs = set(n), []
        for i, blk in enumerate(self.blocks):
            t = blk(t)
            if i in take:
                outs.append(self.norm(t))
        if len(outs) != len(take):
            raise ValueError(f"only {len(outs)} / {len(take)} blocks found")
        if return_class_token:
            return tuple((o[:, 1:], o[:, 0]) for o in outs)
        return tuple(o[:, 1:] for o in outs)


# ---------------------------------------------------------------------------------------------
# DPT head (dpt.py:38-165, util/blocks.py)


class _ResidualConvUnit(nn.Module):
    def __init__(self, f: int, bn: bool):
        super().__init__()
        self.bn = bn
        self.conv1 = nn.Conv2d(f, f, 3, padding=1)
        self.conv2 = nn.Conv2d(f, f, 3, padding=1)
        if bn:
            self.bn1 = nn.BatchNorm2d(f)
            self.bn2 = nn.BatchNorm2d(f)

    def forward(self, x):   # blocks.py:61-86
        y = self.conv1(F.relu(x))
        if self.bn:
            y = self.bn1(y)
        y = self.conv2(F.relu(y))
        if self.bn:
            y = self.bn2(y)
        return y + x


class _FusionBlock(nn.Module):
    def __init__(self, f: int, bn: bool):
        super().__init__()
        self.out_conv = nn.Conv2d(f, f, 1)
        self.resConfUnit1 = _ResidualConvUnit(f, bn)
        self.resConfUnit2 = _ResidualConvUnit(f, bn)

    def forward(self, *xs, size=None):   # blocks.py:122-148
        out = xs[0]
        if len(xs) == 2:
            out = out + self.resConfUnit1(xs[1])
        out = self.resConfUnit2(out)
        if size is None:
            out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
        else:
            out = F.interpolate(out, size=size, mode="bilinear", align_corners=True)
        return self.out_conv(out)


class DPTHead(nn.Module):
    def __init__(self, in_channels: int, features: int = 256, use_bn: bool = False,
                 out_channels: Sequence[int] = (256, 512, 1024, 1024), use_clstoken: bool = False):
        super().__init__()
        oc = list(out_channels)
        self.use_clstoken = use_clstoken
        self.projects = nn.ModuleList([nn.Conv2d(in_channels, c, 1) for c in oc])
        self.resize_layers = nn.ModuleList([
            nn.ConvTranspose2d(oc[0], oc[0], kernel_size=4, stride=4),
            nn.ConvTranspose2d(oc[1], oc[1], kernel_size=2, stride=2),
            nn.Identity(),
            nn.Conv2d(oc[3], oc[3], kernel_size=3, stride=2, padding=1),
        ])
        if use_clstoken:
            self.readout_projects = nn.ModuleList(
                [nn.Sequential(nn.Linear(2 * in_channels, in_channels), nn.GELU()) for _ in oc])
        s = nn.Module()
        for i, c in enumerate(oc):
            setattr(s, f"layer{i + 1}_rn", nn.Conv2d(c, features, 3, padding=1, bias=False))
        for i in range(1, 5):
            setattr(s, f"refinenet{i}", _FusionBlock(features, use_bn))
        s.output_conv1 = nn.Conv2d(features, features // 2, 3, padding=1)
        s.output_conv2 = nn.Sequential(nn.Conv2d(features // 2, 32, 3, padding=1), nn.ReLU(True),
                                       nn.Conv2d(32, 1, 1), nn.ReLU(True), nn.Identity())
        self.scratch = s

    def forward(self, feats, patch_h: int, patch_w: int):   # dpt.py:128-165
        layers = []
        for i, (x, cls) in enumerate(feats):
            if self.use_clstoken:
                x = self.readout_projects[i](torch.cat((x, cls.unsqueeze(1).expand_as(x)), -1))
            x = x.permute(0, 2, 1).reshape(x.shape[0], x.shape[-1], patch_h, patch_w)
            layers.append(self.resize_layers[i](self.projects[i](x)))
        s = self.scratch
        l1, l2, l3, l4 = (getattr(s, f"layer{i + 1}_rn")(x) for i, x in enumerate(layers))
        p = s.refinenet4(l4, size=l3.shape[2:])
        p = s.refinenet3(p, l3, size=l2.shape[2:])
        p = s.refinenet2(p, l2, size=l1.shape[2:])
        p = s.refinenet1(p, l1)
        out = s.output_conv1(p)
        out = F.interpolate(out, (int(patch_h * 14), int(patch_w * 14)), mode="bilinear", align_corners=False)
        return s.output_conv2(out)


# ---------------------------------------------------------------------------------------------
# the model and its resize rule


def _multiple_of(x: float, m: int, min_val: int = 0) -> int:
    # util/transform.py:51-60 (np.round: halves to even)
    y = int(np.round(x / m) * m)
    if y < min_val:
        y = int(np.ceil(x / m) * m)
    return y


def resize_target(h: int, w: int, input_size_width: int = 518, input_size_height: int = 518) -> Tuple[int, int]:
    """(final_h, final_w) of image2tensor (dpt.py:197-229): keep the aspect ratio, scale so both
    sides reach the requested size ('lower_bound'), round to multiples of 14; portrait inputs
    swap the requested width and height."""
    if h > w:
        input_size_width, input_size_height = input_size_height, input_size_width
    sh, sw = input_size_height / h, input_size_width / w
    if sw > sh:
        sh = sw
    else:
        sw = sh
    return _multiple_of(sh * h, 14, input_size_height), _multiple_of(sw * w, 14, input_size_width)


class DepthAnythingV2(nn.Module):
    """dpt.py:168-238 under the reference's constructor and state-dict names."""

    def __init__(self, encoder: str = "vitl", features: int = 256, out_channels=(256, 512, 1024, 1024),
                 use_bn: bool = False, use_clstoken: bool = False):
        super().__init__()
        if encoder not in _VIT:
            raise ValueError(f"unknown ViT encoder {encoder!r}")
        self.encoder = encoder
        self.intermediate_layer_idx = INTERMEDIATE_LAYERS
        self.pretrained = DINOv2(encoder)
        self.depth_head = DPTHead(self.pretrained.embed_dim, features, use_bn, out_channels, use_clstoken)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        ph, pw = x.shape[-2] // 14, x.shape[-1] // 14
        feats = self.pretrained.get_intermediate_layers(x, self.intermediate_layer_idx[self.encoder], True)
        return F.relu(self.depth_head(feats, ph, pw)).squeeze(1)

    def image2tensor(self, raw_image: torch.Tensor, input_size_width: int = 518, input_size_height: int = 518):
        h, w = raw_image.shape[-2], raw_image.shape[-1]
        fh, fw = resize_target(h, w, input_size_width, input_size_height)
        image = F.interpolate(raw_image, (fh, fw), mode="bicubic", align_corners=False)
        for i, (m, s) in enumerate(zip(IMAGENET_MEAN, IMAGENET_STD)):
            image[:, i].sub_(m).div_(s)
        return image, (h, w), (fh, fw)

    @torch.no_grad()
    def infer_image(self, raw_image: torch.Tensor, input_size_width: int = 518, input_size_height: int = 518):
        """[B, 3, H, W] images in [0, 1] -> [B, 1, H, W] relative inverse depth (dpt.py:188-195)."""
        image, (h, w), _ = self.image2tensor(raw_image, input_size_width, input_size_height)
        depth = self.forward(image)
        return F.interpolate(depth.unsqueeze(1), (h, w), mode="bilinear", align_corners=False)


def get_depth_anything_v2(checkpoint_path: Optional[str] = "weights/depth_anything_v2_vitl.pth",
                          encoder: Optional[str] = None, map_location="cpu") -> DepthAnythingV2:
    """depth_anything_v2/__init__.py:8-38: the encoder from the argument or the file name
    (vitl when neither names one), then the checkpoint, loaded weights-only and strictly
    (``checkpoint_path=None``: the architecture only, for seeded weights)."""
    if encoder not in (None, "vits", "vitb", "vitl", "vitg"):
        raise ValueError("Select a valid ViT encoder")
    if encoder is None:
        name = checkpoint_path or ""
        encoder = next((e for e in ("vits", "vitb", "vitl", "vitg") if e in name), None)
        if encoder is None:
            print("Could not infer the ViT encoder from the checkpoint path. Using 'vitl' as default.")
            encoder = "vitl"
    model = DepthAnythingV2(**MODEL_CONFIGS[encoder])
    if checkpoint_path is not None:
        sd = torch.load(checkpoint_path, map_location=map_location, weights_only=True)
        model.load_state_dict(sd["state_dict"] if "state_dict" in sd else sd)
    return model


# ---------------------------------------------------------------------------------------------
# the harnesses' calls


# test.py:191-194 and test_mapreduce_v2.py:124-143 (the latter adds "monkaa")
INPUT_WIDTH = {"kitti2012": 1372, "kitti2015": 1372, "eth3d": 518, "middlebury": 518 * 2, "middlebury2021": 1372,
               "booster": 518 * 2, "layeredflow": 952, "monkaa": 960}
INPUT_HEIGHT = {"kitti2012": 518, "kitti2015": 518, "eth3d": 518, "middlebury": 518 * 2, "middlebury2021": 770,
                "booster": 756, "layeredflow": 532, "monkaa": 544}
_TEST_SETS = set(INPUT_WIDTH) - {"monkaa"}   # test.py's dicts lack monkaa


def mono_pair_test(model: DepthAnythingV2, im2: torch.Tensor, im3: torch.Tensor, dataset: str):
    """test.py:189-199: both views through infer_image at the dataset's input size, then
    min-max normalised jointly (no epsilon).  Returns ([1,1,H,W], [1,1,H,W])."""
    w = INPUT_WIDTH.get(dataset, 518) if dataset in _TEST_SETS else 518
    h = INPUT_HEIGHT.get(dataset, 518) if dataset in _TEST_SETS else 518
    d = model.infer_image(torch.cat([im2, im3], 0), input_size_width=w, input_size_height=h)
    d = (d - d.min()) / (d.max() - d.min())
    return d[0:1], d[1:2]


def mono_pair_mapreduce(model: DepthAnythingV2, im2: torch.Tensor, im3: torch.Tensor, dataset: str) -> torch.Tensor:
    """test_mapreduce_v2.py:113-160: the input size at least the image's, rounded up to a
    multiple of 14; joint min-max with +1e-8.  Returns [2, 1, H, W]."""
    w = int(math.ceil(max(INPUT_WIDTH.get(dataset, 518), im2.shape[-1]) / 14.0) * 14)
    h = int(math.ceil(max(INPUT_HEIGHT.get(dataset, 518), im2.shape[-2]) / 14.0) * 14)
    d = model.infer_image(torch.cat([im2, im3], 0), input_size_width=w, input_size_height=h)
    return (d - d.min()) / (d.max() - d.min() + 1e-8)


# Seeded weights drive the DPT head's last conv negative everywhere, so its ReLU would output
# an all-zero map (and the joint min-max a 0 / 0): the seeded producer raises that bias.
SEEDED_LAST_BIAS = 0.3


def seeded_model(encoder: str = "vits", seed: int = 0) -> DepthAnythingV2:
    """The producer on seeded weights (synth.seeded_state_dict) with the head's last bias at
    SEEDED_LAST_BIAS: the weights of tests/golden/dav2.npz (make_golden.DAV2_LAST_BIAS)."""
    from . import synth

    m = DepthAnythingV2(**MODEL_CONFIGS[encoder])
    synth.load_seeded_weights(m, seed)
    with torch.no_grad():
        m.depth_head.scratch.output_conv2[2].bias.fill_(SEEDED_LAST_BIAS)
    return m.eval()


def load_for_harness(args, device) -> Optional[DepthAnythingV2]:
    """The CLIs' mono model (test.py:133-138): ``--monomodel DAv2`` with ``--loadmonomodel``
    a DAv2 checkpoint (or ``seeded``: :func:`seeded_model` for ``--vit_encoder``, as no
    checkpoint is reachable offline).  None without ``--loadmonomodel``: the precomputed maps
    (``--mono_tag``) are used instead."""
    if args.monomodel != "DAv2" or not args.loadmonomodel:
        return None
    if args.loadmonomodel == "seeded":
        m = seeded_model(args.vit_encoder)
    else:
        m = get_depth_anything_v2(args.loadmonomodel, encoder=args.vit_encoder)
    return m.to(device).eval()
