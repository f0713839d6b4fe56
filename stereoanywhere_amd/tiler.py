"""Host-side tiler for high-resolution pairs (configs 3 and 5: Middlebury-H, Booster).

Mirrors the reference's mapreduce_v2 package so results stitch identically:
  * ``TileWrapper`` (tile_wrapper.py:52-362) — same constructor (square ``tile_size`` or
    rectangular ``tile_width``/``tile_height``, ``overlap`` default 256, ``batch_tiles``,
    ``device``) and forward (``mixed_precision``, ``global_guidance``, ``guidance_weight``).
    Tile grid with stride ``tile - overlap`` and the last tile pushed back inside the image,
    which can emit the same rectangle twice (101-120); per tile: replicate-pad to a multiple
    of 32 (left/top get pad//2, 226-236), run the model, negate (``_canonicalize_output``,
    188-206), unpad, optionally blend with the global guidance map, and accumulate with the
    clamped sin·sin weight (36-49, 328-362); stitched / weight where weight > 0 (185).  An
    image that fits one tile runs the model directly (151-153) and ignores the guidance.
  * ``MapReduceInference`` (tiled_inference.py:25-336) — uint8 HxWx3 images -> /255 ->
    bilinear ``iscale`` resize -> optional low-resolution global-guidance pass -> tiler ->
    nearest ``oscale`` resize and ``post_scale``.
  * ``tiling_for`` / ``select_tiling_parameters`` — the rounding rules of MapReduceInference
    (56-99) and the VRAM heuristic of memory_utils.py:34-57.
  * ``to_uint8_image`` — the harness's clip / x255 / truncating cast
    (test_mapreduce_v2.py:163-175).
Duplicate rectangles of the enumeration run once and are accumulated once per occurrence,
in the reference's order.
Multi-GPU: with ``rank``/``world`` set, rank r processes unique tiles r, r+world, ...; the partial
stitched and weight maps are summed with one all_reduce (RCCL over xGMI) — the tiled
path's only exchange.

The model computes fp32 throughout: ``mixed_precision`` is accepted for API compatibility
and, like the reference's tiled path (tile_wrapper.py:135 pops it from **kwargs, so the
keyword argument never reaches autocast), does not change the arithmetic.
"""
from __future__ import annotations

import hashlib
import math
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import ops


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


@dataclass
class TilingParameters:
    tile_size: int
    overlap: int


def select_tiling_parameters(default_tile: int = 1024, default_overlap: int = 256, min_tile: int = 256,
                             device: int = 0) -> TilingParameters:
    """memory_utils.py:34-57: tile side from the free device memory (an MI355X has 288 GB,
    so the default 1024 / 256); without a GPU the minimum tile."""
    if not torch.cuda.is_available():
        return TilingParameters(min_tile, min_tile // 4)
    torch.cuda.synchronize(device)
    stats = torch.cuda.memory_stats(device)
    # Deliberate parity with the reference (memory_utils.py:27-28): it reads the keys
    # "reserved_bytes.all" / "allocated_bytes.all", which torch.cuda.memory_stats() does not have
    # (its keys are "reserved_bytes.all.current" etc.), so `used` is always 0 and the tile size
    # follows the total memory.  Kept so the tiling, and with it the output, equals the
    # reference's; on an MI355X (288 GB) either reading gives the default 1024 / 256.
    used = max(stats.get("reserved_bytes.all", 0), stats.get("allocated_bytes.all", 0))
    free_mb = max(torch.cuda.get_device_properties(device).total_memory - used, 0) / 2 ** 20
    if free_mb <= 0:
        return TilingParameters(min_tile, min_tile // 4)
    tile = (max(min_tile, 512) if free_mb < 2048 else max(min_tile, 768) if free_mb < 4096
            else max(min_tile, 896) if free_mb < 6144 else default_tile)
    return TilingParameters(tile, min(tile // 4, default_overlap))


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


def _hip_tiles(*ts) -> bool:
    """The GPU gather / stitch (ops.tile_gather_pad / tile_stitch) take float32 CUDA images of batch 1;
    anything else (CPU tensors: the harness tests' mock models) keeps the torch ops."""
    return all(t is None or (t.is_cuda and t.dtype == torch.float32 and t.dim() == 4 and t.shape[0] == 1)
               for t in ts) and ts[0] is not None


def guidance_blend(disp: torch.Tensor, guide: torch.Tensor, weight: float) -> torch.Tensor:
    """tile_wrapper.py:347-357: confidence = 1 - |d - g| / (max|d - g| + 1e-6) over the
    tile; the guidance pulls the tile by weight * confidence."""
    diff = torch.abs(disp - guide)
    infl = weight * (1.0 - diff / (torch.max(diff) + 1e-6))
    return (1.0 - infl) * disp + infl * guide


def pad32(h: int, w: int):
    ph = (((h // 32) + 1) * 32 - h) % 32
    pw = (((w // 32) + 1) * 32 - w) % 32
    return [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2]


def canonicalize(output) -> torch.Tensor:
    if isinstance(output, (tuple, list)):
        output = output[0]
    if not isinstance(output, torch.Tensor):
        raise TypeError("Model output must be a tensor or tuple/list of tensors")
    if output.dim() == 3:
        output = output.unsqueeze(1)
    if output.dim() != 4:
        raise ValueError("Model output must be BCHW")
    if output.shape[1] != 1:
        raise ValueError("Disparity tensor must have a single channel")
    return -output


class TileWrapper(torch.nn.Module):
    """tile_wrapper.py:52-362 (constructor 55-93: rectangular tiles when both sides are
    given and positive, else square ``tile_size``; same ValueErrors)."""

    def __init__(self, model, tile_size: Optional[int] = None, tile_width: Optional[int] = None,
                 tile_height: Optional[int] = None, overlap: int = 256, batch_tiles: bool = False,
                 device: Optional[torch.device] = None, *, rank: int = 0, world: int = 1):
        super().__init__()
        if tile_width is not None and tile_height is not None and tile_width > 0 and tile_height > 0:
            self.tile_width, self.tile_height, self.use_rectangular = tile_width, tile_height, True
        else:
            if tile_size is None or tile_size <= 0:
                raise ValueError("tile_size must be > 0 when not using rectangular tiles")
            self.tile_width = self.tile_height = tile_size
            self.use_rectangular = False
        if overlap < 0:
            raise ValueError("overlap must be >= 0")
        if overlap >= min(self.tile_width, self.tile_height):
            raise ValueError("overlap must be smaller than the minimum of tile_width and tile_height")
        self.model = model
        self.overlap = overlap
        self.batch_tiles = batch_tiles
        self._device_override = device
        self.rank, self.world = rank, world

    @property
    def device(self) -> torch.device:
        if self._device_override is not None:
            return self._device_override
        return next(self.model.parameters()).device

    def _enumerate_tiles(self, height: int, width: int) -> List[TileSpec]:
        return enumerate_tiles(height, width, self.tile_height, self.tile_width, self.overlap)

    def _run(self, left, right, ml, mr, args, kw):
        _pad = pad32(*left.shape[-2:])

        def pad(t):
            return None if t is None else F.pad(t, _pad, mode="replicate")
        disp = canonicalize(self.model(pad(left), pad(right), pad(ml), pad(mr), *args, **kw))
        hd, wd = disp.shape[-2:]
        return disp[..., _pad[2]:hd - _pad[3], _pad[0]:wd - _pad[1]]

    def forward(self, left, right, mono_left=None, mono_right=None, *args, mixed_precision: bool = False,
                global_guidance: Optional[torch.Tensor] = None, guidance_weight: float = 0.3, **kw):
        if left.shape != right.shape:
            raise ValueError("Left/right inputs must have identical shape")
        for name, m, ref in (("mono_left", mono_left, left), ("mono_right", mono_right, right)):
            if m is not None and (m.shape[0] != ref.shape[0] or m.shape[-2:] != ref.shape[-2:]):
                raise ValueError(f"{name} must share batch and spatial shape with {name.split('_')[1]} input")
        B, _, H, W = left.shape
        if B != 1:
            raise ValueError("TileWrapper currently supports batch size == 1")
        if H <= self.tile_height and W <= self.tile_width:
            self.last_tile_counts = (1, 1)
            return canonicalize(self.model(left, right, mono_left, mono_right, *args, **kw))
        guide = None
        if global_guidance is not None and guidance_weight > 0:
            guide = global_guidance
            while guide.dim() < 4:   # a bare HxW map (the reference indexes it as BCHW)
                guide = guide.unsqueeze(0)
            if guide.shape[-2:] != (H, W):
                raise ValueError("global_guidance must match the input's spatial shape")
        device = self.device
        tiles = self._enumerate_tiles(H, W)
        # The enumeration can emit one rectangle twice (the last row / column is pushed back
        # inside the image: config 3's 1024-row image gives rows y = 0 and y = 992 both as
        # 0..1024).  Each unique rectangle runs once; the accumulation below still visits the
        # tiles in the reference's order, so a duplicate adds the same d * w again and the
        # stitched sums equal the reference's (tile_wrapper.py:169-185) term for term.
        unique = list(dict.fromkeys(tiles))
        self.last_tile_counts = (len(tiles), len(unique))
        stitched = torch.zeros((1, 1, H, W), device=device, dtype=torch.float32)
        weight = torch.zeros_like(stitched)
        mine = unique[self.rank::self.world]

        def view(t, s):
            return None if t is None else t[:, :, s.y_start:s.y_end, s.x_start:s.x_end]

        hip = _hip_tiles(left, right, mono_left, mono_right) and len({(s.height, s.width) for s in tiles}) == 1
        if self.batch_tiles and mine and hip:
            # the batch cut and replicate-padded on the GPU in one launch per tensor (sa_tile_gather_pad:
            # the torch.cat + F.pad of the branch below, bit for bit)
            th, tw = mine[0].height, mine[0].width
            _pad = pad32(th, tw)
            org = [(s.y_start, s.x_start) for s in mine]

            def gp(t):
                return None if t is None else ops.tile_gather_pad(t.contiguous(), org, th, tw, _pad)
            disp = canonicalize(self.model(gp(left), gp(right), gp(mono_left), gp(mono_right), *args, **kw))
            hd, wd = disp.shape[-2:]
            outs = disp[..., _pad[2]:hd - _pad[3], _pad[0]:wd - _pad[1]]
            if guide is None and outs.device == device and outs.shape[-2:] == (th, tw):
                # the stitching loop below in one launch (sa_tile_stitch), same order, same bits
                slot = {s: i for i, s in enumerate(mine)}
                wgt = blend_weight(th, tw, device).contiguous()
                listed = [(s.y_start, s.x_start, slot[s]) for s in tiles if s in slot]
                ops.tile_stitch(outs, listed, wgt, H, W, self.world == 1, stitched.view(H, W), weight.view(H, W))
                if self.world == 1:
                    return stitched
                import torch.distributed as dist
                both = torch.cat([stitched, weight], 1)
                dist.all_reduce(both)
                stitched, weight = both[:, :1], both[:, 1:]
                return torch.where(weight > 0, stitched / torch.clamp(weight, min=1e-4), stitched)
            outs = list(outs.split(1, 0))
        elif self.batch_tiles and mine:
            # every tile has the same size (tiles are pushed inside the image), so batch them
            outs = self._run(torch.cat([view(left, s) for s in mine]), torch.cat([view(right, s) for s in mine]),
                             None if mono_left is None else torch.cat([view(mono_left, s) for s in mine]),
                             None if mono_right is None else torch.cat([view(mono_right, s) for s in mine]),
                             args, kw)
            outs = list(outs.split(1, 0))
        else:
            outs = [self._run(view(left, s), view(right, s), view(mono_left, s), view(mono_right, s), args, kw)
                    for s in mine]
        done = {}
        for s, d in zip(mine, outs):
            d = d.detach().to(device)
            if d.shape[-2:] != (s.height, s.width):
                raise ValueError("Tile output spatial size mismatch")
            if guide is not None:
                d = guidance_blend(d, view(guide, s).to(d.device, d.dtype), guidance_weight)
            done[s] = d
        wgts = {}
        for s in tiles:
            d = done.get(s)
            if d is None:   # another rank's rectangle
                continue
            wgt = wgts.get((s.height, s.width))
            if wgt is None:
                wgt = wgts[(s.height, s.width)] = blend_weight(s.height, s.width, d.device)[None, None]
            stitched[:, :, s.y_start:s.y_end, s.x_start:s.x_end] += d * wgt
            weight[:, :, s.y_start:s.y_end, s.x_start:s.x_end] += wgt
        if self.world > 1:
            import torch.distributed as dist
            both = torch.cat([stitched, weight], 1)
            dist.all_reduce(both)
            stitched, weight = both[:, :1], both[:, 1:]
        return torch.where(weight > 0, stitched / torch.clamp(weight, min=1e-4), stitched)


_DATASET_PRESET = {"middlebury": "middlebury", "middlebury2014": "middlebury", "middlebury2021": "middlebury",
                   "kitti": "kitti", "kitti2012": "kitti", "kitti2015": "kitti", "sceneflow": "sceneflow",
                   "flyingthings": "sceneflow", "driving": "sceneflow", "monkaa": "sceneflow", "booster": "booster",
                   "monotrap": "monotrap"}


def get_preset(name: str) -> TilePreset:
    """tile_presets.py:131-150."""
    if name not in TILE_PRESETS:
        raise ValueError(f"unknown preset {name!r}; available: {', '.join(TILE_PRESETS)}")
    return TILE_PRESETS[name]


def get_preset_for_dataset(dataset: str) -> TilePreset:
    """tile_presets.py:165-200: first mapping key contained in the (lower-cased) name, in
    the mapping's order; 'default' otherwise."""
    low = dataset.lower()
    for key, name in _DATASET_PRESET.items():
        if key in low:
            return TILE_PRESETS[name]
    return TILE_PRESETS["default"]


def from_preset(model, preset: str, **kw) -> TileWrapper:
    p = TILE_PRESETS[preset]
    tw, th, ov = tiling_for(p.tile_width, p.tile_height, p.overlap)
    return TileWrapper(model, tile_width=tw, tile_height=th, overlap=ov, **kw)


# ------------------------------------------------------------------ uint8 image helpers

def to_uint8_image(t: torch.Tensor) -> np.ndarray:
    """test_mapreduce_v2.py:163-175: [1,3,H,W] float in [0,1] -> HxWx3 uint8, clipped and
    TRUNCATED (astype), not rounded."""
    img = t.detach().cpu().squeeze(0).permute(1, 2, 0).numpy()
    return (np.clip(img, 0.0, 1.0) * 255).astype(np.uint8)


def _area_weights(n_src: int, n_dst: int) -> np.ndarray:
    """Fraction of source cell j inside destination cell i (area resampling, scale >= 1)."""
    s = n_src / n_dst
    w = np.zeros((n_dst, n_src), np.float64)
    for i in range(n_dst):
        a, b = i * s, min((i + 1) * s, n_src)
        for j in range(int(math.floor(a)), int(math.ceil(b))):
            w[i, j] = (min(b, j + 1) - max(a, j)) / s
    return w


def resize_area_u8(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """Area down-sampling of an HxWxC uint8 image, the cv2.resize(INTER_AREA) algorithm the
    guidance pass calls (tiled_inference.py:190-191): each output pixel is the area-weighted
    mean of the source cells it covers.  Exact integer factors average whole blocks and
    round half up (cv2's fast path); other factors round half to even.  cv2 is not installed
    in this image, so this restatement is parity-unpinned against cv2 itself."""
    H, W = img.shape[:2]
    if out_w > W or out_h > H:
        raise ValueError("resize_area_u8 only down-samples")
    x = img.astype(np.float64)
    y = np.einsum("ih,hwc->iwc", _area_weights(H, out_h), x)
    y = np.einsum("jw,iwc->ijc", _area_weights(W, out_w), y)
    fast = H % out_h == 0 and W % out_w == 0
    y = np.floor(y + 0.5) if fast else np.rint(y)
    return np.clip(y, 0, 255).astype(np.uint8)


@dataclass
class TiledInputs:
    left: torch.Tensor
    right: torch.Tensor
    mono_left: Optional[torch.Tensor]
    mono_right: Optional[torch.Tensor]


class MapReduceInference:
    """tiled_inference.py:25-336: uint8 images in, numpy disparity out."""

    def __init__(self, stereo_model: torch.nn.Module, mono_model: Optional[Callable] = None,
                 tile_size: Optional[int] = None, tile_width: Optional[int] = None,
                 tile_height: Optional[int] = None, overlap: Optional[int] = None, batch_tiles: bool = False,
                 mixed_precision: bool = False, clear_cache: bool = False, auto_tiling: bool = True,
                 use_global_guidance: bool = False, guidance_scale: float = 2.0, guidance_weight: float = 0.3,
                 *, rank: int = 0, world: int = 1) -> None:
        self.stereo_model = stereo_model
        self.mono_model = mono_model
        self.mixed_precision = mixed_precision
        self.clear_cache = clear_cache
        self.use_global_guidance = use_global_guidance
        self.guidance_scale = guidance_scale
        self.guidance_weight = guidance_weight
        self._guidance_cache = {}
        if tile_width is not None and tile_height is not None and tile_width > 0 and tile_height > 0:
            if overlap is None:
                overlap = select_tiling_parameters().overlap
            tw, th, ov = tiling_for(tile_width, tile_height, overlap)
            self.tile_wrapper = TileWrapper(stereo_model, tile_width=tw, tile_height=th, overlap=ov,
                                            batch_tiles=batch_tiles, rank=rank, world=world)
        else:
            if tile_size is None or overlap is None:
                p = select_tiling_parameters()
                tile_size, overlap = p.tile_size, p.overlap
            ts = _up32(tile_size)
            ov = int(min(ts - 32, (overlap + 31) // 32 * 32)) if overlap else 0
            self.tile_wrapper = TileWrapper(stereo_model, tile_size=ts, overlap=ov, batch_tiles=batch_tiles,
                                            rank=rank, world=world)

    @staticmethod
    def _to_tensor(img: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).float().unsqueeze(0) / 255.0

    def _prepare_inputs(self, left_img, right_img, iscale, mono_size, device, dtype, mono_pair=None) -> TiledInputs:
        """tiled_inference.py:101-143."""
        target = (round(left_img.shape[0] / iscale), round(left_img.shape[1] / iscale))
        lt, rt = self._to_tensor(left_img), self._to_tensor(right_img)

        def rs(t):
            return F.interpolate(t, size=target, mode="bilinear", align_corners=False)
        left = (rs(lt) if iscale != 1.0 else lt).to(device=device, dtype=dtype)
        right = (rs(rt) if iscale != 1.0 else rt).to(device=device, dtype=dtype)
        ml = mr = None
        if mono_pair is not None:
            ml, mr = (rs(m).to(device=device, dtype=dtype) for m in mono_pair)
        elif self.mono_model is not None:
            ml = rs(self.mono_model(lt.to(device=device, dtype=dtype), mono_size)).to(device=device, dtype=dtype)
            mr = rs(self.mono_model(rt.to(device=device, dtype=dtype), mono_size)).to(device=device, dtype=dtype)
        return TiledInputs(left, right, ml, mr)

    def _compute_global_guidance(self, left_img, right_img, mono_pair, device, dtype,
                                 verbose: bool = False) -> Optional[np.ndarray]:
        """tiled_inference.py:145-228: one untiled pass at 1/guidance_scale (area down-sampled
        uint8 images, iters=32), bilinear back to full size and multiplied by the scale;
        cached by the left image's bytes."""
        if not self.use_global_guidance:
            return None
        key = hashlib.md5(left_img.tobytes()).hexdigest()
        if key in self._guidance_cache:
            return self._guidance_cache[key]
        h, w = left_img.shape[:2]
        th, tw = int(h / self.guidance_scale), int(w / self.guidance_scale)
        lt = self._to_tensor(resize_area_u8(left_img, tw, th)).to(device=device, dtype=dtype)
        rt = self._to_tensor(resize_area_u8(right_img, tw, th)).to(device=device, dtype=dtype)
        ml = mr = None
        if mono_pair is not None:
            ml, mr = (F.interpolate(m, size=(th, tw), mode="bilinear", align_corners=False) for m in mono_pair)
        elif self.mono_model is not None:
            ml, mr = self.mono_model(lt, (th, tw)), self.mono_model(rt, (th, tw))
        with torch.no_grad():
            low = canonicalize(self.stereo_model(lt, rt, ml, mr, iters=32, test_mode=True)).float()
        # cv2.resize(INTER_LINEAR) up-sampling == half-pixel bilinear with edge clamping
        g = F.interpolate(low.cpu(), size=(h, w), mode="bilinear", align_corners=False)[0, 0].numpy()
        g = g * np.float32(self.guidance_scale)
        self._guidance_cache[key] = g
        if verbose:
            print(f"[Guidance] computed and cached guidance: {g.shape}")
        return g

    def infer(self, left_img: np.ndarray, right_img: np.ndarray, *, iscale: float = 1.0, oscale: float = 1.0,
              mono_size: Tuple[int, int] = (518, 518), post_scale: float = 1.0, verbose: bool = False,
              mono_pair: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
              global_guidance: Optional[np.ndarray] = None, guidance_weight: float = 0.3, **kwargs) -> np.ndarray:
        """tiled_inference.py:230-336."""
        p = next(self.stereo_model.parameters())
        device, dtype = p.device, p.dtype
        inputs = self._prepare_inputs(left_img, right_img, iscale, mono_size, device, dtype, mono_pair=mono_pair)
        if self.use_global_guidance and global_guidance is None:
            global_guidance = self._compute_global_guidance(left_img, right_img, mono_pair, device, dtype, verbose)
        guide = None
        if global_guidance is not None:
            guide = (torch.from_numpy(global_guidance) if isinstance(global_guidance, np.ndarray)
                     else global_guidance).float()
            target = tuple(inputs.left.shape[-2:])
            if tuple(guide.shape[-2:]) != target:
                guide = guide[None, None] if guide.dim() == 2 else guide
                # the reference rescales by target_w / guide_w AFTER resizing, i.e. by 1
                # (tiled_inference.py:292-293): values are kept as given
                guide = F.interpolate(guide, size=target, mode="bilinear", align_corners=False)
            guide = guide.to(device=device, dtype=dtype)
            if guidance_weight == 0.3:   # the default -> the instance's weight (298-299)
                guidance_weight = self.guidance_weight
        with torch.no_grad():
            disp = self.tile_wrapper(inputs.left, inputs.right, inputs.mono_left, inputs.mono_right,
                                     mixed_precision=self.mixed_precision, global_guidance=guide,
                                     guidance_weight=guidance_weight, **kwargs)
        disp = disp.squeeze(0).squeeze(0).float().cpu().numpy()
        if oscale != iscale or post_scale != 1.0:
            target = (round(left_img.shape[0] / oscale), round(left_img.shape[1] / oscale))
            d = F.interpolate(torch.from_numpy(disp)[None, None], size=target, mode="nearest")
            disp = d.squeeze().numpy() * (iscale / oscale) * post_scale
        else:
            disp *= post_scale
        if self.clear_cache and torch.cuda.is_available():
            torch.cuda.empty_cache()
        return disp
