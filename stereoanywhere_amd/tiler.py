"""Host-side tiler for high-resolution pairs (configs 3 and 5: Middlebury-H, Booster).

Mirrors the reference's mapreduce_v2 tiler so results stitch identically:
  * ``TileWrapper`` — tile grid with stride ``tile - overlap`` and the last tile pushed
    back inside the image, which can emit the same rectangle twice (tile_wrapper.py:101-120);
    per tile: replicate-pad to a multiple of 32 (left/top get pad//2, 226-236), run the
    model with ``test_mode=True``, negate (``_canonicalize_output``, 188-206), unpad, and
    accumulate with the clamped sin·sin blend weight (36-49, 328-362); stitched / weight
    where weight > 0 (185).  An image that fits one tile runs the model directly (151-153).
  * ``tiling_for`` — the preset / rounding rules of MapReduceInference (tiled_inference.py:
    52-99): tile sides rounded UP to multiples of 32, overlap rounded up to 32 and capped at
    min(tile) - 32.
Multi-GPU: with ``rank``/``world`` set, rank r processes tiles r, r+world, ...; the partial
stitched and weight maps are summed with one all_reduce (RCCL over xGMI) — the tiled
path's only exchange.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class TileSpec:
    y_start: int
    y_end: int
    x_start: int
    x_end: int

    @property
    def height(self) -> int:
        return self.y_end - self.y_start

    @property
    def width(self) -> int:
        return self.x_end - self.x_start


@dataclass(frozen=True)
class TilePreset:
    name: str
    tile_width: int
    tile_height: int
    overlap: int


# tile_presets.py:37-127 (the sizes the benchmark configs use)
TILE_PRESETS = {p.name: p for p in [
    TilePreset("default", 448, 448, 96), TilePreset("middlebury", 672, 1120, 112),
    TilePreset("kitti", 1344, 448, 128), TilePreset("sceneflow", 448, 448, 112),
    TilePreset("booster", 1120, 896, 224), TilePreset("monotrap", 800, 600, 96),
    TilePreset("small_image", 1024, 1024, 64), TilePreset("large_image", 512, 512, 64),
    TilePreset("low_memory", 512, 384, 48), TilePreset("high_memory", 1280, 960, 128),
]}


def _up32(v: int) -> int:
    return int(max(32, (v + 31) // 32 * 32))


def tiling_for(tile_width: int, tile_height: int, overlap: int) -> Tuple[int, int, int]:
    """MapReduceInference's rounding (tiled_inference.py:56-69): (tile_w, tile_h, overlap)."""
    tw, th = _up32(tile_width), _up32(tile_height)
    ov = int(min(min(tw, th) - 32, (overlap + 31) // 32 * 32)) if overlap else 0
    return tw, th, ov


def enumerate_tiles(height: int, width: int, tile_h: int, tile_w: int, overlap: int) -> List[TileSpec]:
    sy, sx = tile_h - overlap, tile_w - overlap
    tiles = []
    y = 0
    while y < height:
        y1 = min(y + tile_h, height)
        y0 = max(0, y1 - tile_h)
        x = 0
        while x < width:
            x1 = min(x + tile_w, width)
            x0 = max(0, x1 - tile_w)
            tiles.append(TileSpec(y0, y1, x0, x1))
            x += sx
        y += sy
    return tiles


def blend_weight(height: int, width: int, device) -> torch.Tensor:
    """sin(pi*y) * sin(pi*x) on linspace(0, 1) grids, clamped at 1e-4."""
    y = torch.linspace(0, 1, height, device=device)
    x = torch.linspace(0, 1, width, device=device)
    gy, gx = torch.meshgrid(y, x, indexing="ij")
    w = torch.sin(torch.pi * torch.clamp(gy, 0, 1)) * torch.sin(torch.pi * torch.clamp(gx, 0, 1))
    return torch.clamp(w, min=1e-4)


def pad32(h: int, w: int):
    ph = (((h // 32) + 1) * 32 - h) % 32
    pw = (((w // 32) + 1) * 32 - w) % 32
    return [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2]


def canonicalize(output) -> torch.Tensor:
    if isinstance(output, (tuple, list)):
        output = output[0]
    if output.dim() == 3:
        output = output.unsqueeze(1)
    if output.dim() != 4 or output.shape[1] != 1:
        raise ValueError("model output must be a [B,1,H,W] disparity tensor")
    return -output


class TileWrapper(torch.nn.Module):
    def __init__(self, model, tile_width: int, tile_height: int, overlap: int, batch_tiles: bool = False,
                 rank: int = 0, world: int = 1):
        super().__init__()
        if tile_width <= 0 or tile_height <= 0 or overlap < 0 or overlap >= min(tile_width, tile_height):
            raise ValueError("invalid tile geometry")
        self.model = model
        self.tile_width, self.tile_height, self.overlap = tile_width, tile_height, overlap
        self.batch_tiles = batch_tiles
        self.rank, self.world = rank, world

    def _run(self, left, right, ml, mr, kw):
        _pad = pad32(*left.shape[-2:])

        def pad(t):
            return None if t is None else F.pad(t, _pad, mode="replicate")
        disp = canonicalize(self.model(pad(left), pad(right), pad(ml), pad(mr), **kw))
        hd, wd = disp.shape[-2:]
        return disp[..., _pad[2]:hd - _pad[3], _pad[0]:wd - _pad[1]]

    def forward(self, left, right, mono_left=None, mono_right=None, **kw):
        kw.setdefault("test_mode", True)
        if left.shape != right.shape:
            raise ValueError("left/right inputs must have identical shape")
        B, _, H, W = left.shape
        if B != 1:
            raise ValueError("TileWrapper supports batch size 1 (tile_wrapper.py:148-149)")
        if H <= self.tile_height and W <= self.tile_width:
            return canonicalize(self.model(left, right, mono_left, mono_right, **kw))
        tiles = enumerate_tiles(H, W, self.tile_height, self.tile_width, self.overlap)
        stitched = torch.zeros((1, 1, H, W), device=left.device, dtype=torch.float32)
        weight = torch.zeros_like(stitched)
        mine = tiles[self.rank::self.world]

        def view(t, s):
            return None if t is None else t[:, :, s.y_start:s.y_end, s.x_start:s.x_end]

        if self.batch_tiles and mine:
            # every tile has the same size (tiles are pushed inside the image), so batch them
            outs = self._run(torch.cat([view(left, s) for s in mine]), torch.cat([view(right, s) for s in mine]),
                             None if mono_left is None else torch.cat([view(mono_left, s) for s in mine]),
                             None if mono_right is None else torch.cat([view(mono_right, s) for s in mine]), kw)
            outs = list(outs.split(1, 0))
        else:
            outs = [self._run(view(left, s), view(right, s), view(mono_left, s), view(mono_right, s), kw)
                    for s in mine]
        for s, d in zip(mine, outs):
            wgt = blend_weight(s.height, s.width, d.device)[None, None]
            stitched[:, :, s.y_start:s.y_end, s.x_start:s.x_end] += d.float() * wgt
            weight[:, :, s.y_start:s.y_end, s.x_start:s.x_end] += wgt
        if self.world > 1:
            import torch.distributed as dist
            both = torch.cat([stitched, weight], 1)
            dist.all_reduce(both)
            stitched, weight = both[:, :1], both[:, 1:]
        return torch.where(weight > 0, stitched / torch.clamp(weight, min=1e-4), stitched)


def from_preset(model, preset: str, **kw) -> TileWrapper:
    p = TILE_PRESETS[preset]
    tw, th, ov = tiling_for(p.tile_width, p.tile_height, p.overlap)
    return TileWrapper(model, tw, th, ov, **kw)
