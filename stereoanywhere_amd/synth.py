"""Seeded synthetic stereo pairs and seeded model weights.

No dataset or checkpoint is reachable from this pipeline, so
every parity test and every bench run feeds:

* weights drawn from ``numpy.random.default_rng([seed, crc32(name)])`` per
  state-dict entry, so the same tensor gets the same values on any machine and
  in any model that uses the reference's parameter names
  (reference: models/stereoanywhere/stereoanywhere.py:52-76);
* stereo pairs built as BASELINE.md §3 describes: 4-octave value noise for the
  left view, a smooth disparity field in [0.1·D, 0.9·D] px, the right view
  sampled from the left at x + d (border clamp), and the mono maps set to the
  min-max-normalised disparity (the global maximum is exactly 1.0, which lands
  in no mask bin — SURVEY.md Appendix A.3).

Everything is numpy float64 arithmetic cast to float32 at the end, so the bytes
are identical here and on the GPU box.
"""
from __future__ import annotations

import hashlib
import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

# ----------------------------------------------------------------------------
# weights


def _conv_fans(shape: Tuple[int, ...]) -> Tuple[int, int]:
    rf = int(np.prod(shape[2:])) if len(shape) > 2 else 1
    return shape[1] * rf, shape[0] * rf


def seeded_state_dict(template: Dict[str, "np.ndarray"], seed: int = 0) -> Dict[str, np.ndarray]:
    """Return {name: float32 array} for every entry of ``template`` (name -> shape).

    * conv weights of the two encoders (``fnet.``/``cnet.``): N(0, sqrt(2/fan_out)),
      the reference's kaiming_normal(fan_out) init (extractor.py:152-158, 249-255);
    * every other conv / linear weight and bias: U(-1/sqrt(fan_in), 1/sqrt(fan_in)),
      torch's default Conv init;
    * BatchNorm affine and running statistics: perturbed around (1, 0, 0, 1) so the
      eval-mode normalisation is exercised, ``num_batches_tracked`` = 0.
    """
    shapes = {k: tuple(v) for k, v in template.items()}
    out: Dict[str, np.ndarray] = {}
    for name, shape in shapes.items():
        # ResidualBlock registers one norm module twice (as norm3 and downsample.1,
        # extractor.py:19-45); both names must carry the same values.
        key = name.replace(".norm3.", ".downsample.1.")
        rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            out[name] = np.zeros(shape, dtype=np.int64)
            continue
        if leaf == "weight" and len(shape) >= 2:
            fan_in, fan_out = _conv_fans(shape)
            if name.startswith(("fnet.", "cnet.")):
                w = rng.standard_normal(shape) * np.sqrt(2.0 / fan_out)
            else:
                b = 1.0 / np.sqrt(fan_in)
                w = rng.uniform(-b, b, shape)
            out[name] = w.astype(np.float32)
            continue
        if leaf == "bias":
            wname = name[: -len("bias")] + "weight"
            if wname in shapes and len(shapes[wname]) >= 2:
                fan_in, _ = _conv_fans(shapes[wname])
                b = 1.0 / np.sqrt(fan_in)
                out[name] = rng.uniform(-b, b, shape).astype(np.float32)
            else:  # norm bias
                out[name] = rng.uniform(-0.05, 0.05, shape).astype(np.float32)
            continue
        if leaf in ("weight", "gamma"):  # norm scale, ViT LayerScale
            out[name] = rng.uniform(0.9, 1.1, shape).astype(np.float32)
        elif leaf in ("cls_token", "pos_embed", "mask_token", "register_tokens"):
            # ViT embeddings (depth_anything_v2/dinov2.py:109-114, init 230-235): N(0, 0.02)
            out[name] = (rng.standard_normal(shape) * 0.02).astype(np.float32)
        elif leaf == "running_mean":
            out[name] = rng.uniform(-0.05, 0.05, shape).astype(np.float32)
        elif leaf == "running_var":
            out[name] = rng.uniform(0.9, 1.1, shape).astype(np.float32)
        else:
            raise KeyError(f"no seeded rule for parameter {name} {shape}")
    return out


def load_seeded_weights(module, seed: int = 0) -> None:
    """Fill a torch module's state dict in place with :func:`seeded_state_dict`."""
    import torch

    sd = module.state_dict()
    vals = seeded_state_dict({k: tuple(v.shape) for k, v in sd.items()}, seed)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=True)


# ----------------------------------------------------------------------------
# stereo pairs


def _upsample_bilinear(grid: np.ndarray, H: int, W: int) -> np.ndarray:
    """align_corners=True bilinear upsampling of a 2-D float64 grid (no reductions)."""
    gh, gw = grid.shape
    ys = np.linspace(0.0, gh - 1, H)
    xs = np.linspace(0.0, gw - 1, W)
    y0 = np.clip(np.floor(ys).astype(np.int64), 0, gh - 1)
    x0 = np.clip(np.floor(xs).astype(np.int64), 0, gw - 1)
    y1 = np.minimum(y0 + 1, gh - 1)
    x1 = np.minimum(x0 + 1, gw - 1)
    wy = (ys - y0)[:, None]
    wx = (xs - x0)[None, :]
    top = grid[y0][:, x0] * (1 - wx) + grid[y0][:, x1] * wx
    bot = grid[y1][:, x0] * (1 - wx) + grid[y1][:, x1] * wx
    return top * (1 - wy) + bot * wy


def _value_noise(rng: np.random.Generator, H: int, W: int, octaves=(1, 2, 4, 8)) -> np.ndarray:
    acc = np.zeros((H, W))
    for s in octaves:
        g = rng.random((max(2, H // s), max(2, W // s)))
        acc = acc + _upsample_bilinear(g, H, W)
    return acc / len(octaves)


def synthetic_pair(H: int, W: int, max_disp: float, seed: int) -> Dict[str, np.ndarray]:
    """One synthetic pair: left/right [3,H,W] in [0,1], mono L/R [1,H,W], disparity [H,W]."""
    rng = np.random.default_rng([1000 + seed, H, W])
    left = np.stack([_value_noise(rng, H, W) for _ in range(3)], 0)
    dgrid = rng.random((max(2, H // 32), max(2, W // 32)))
    disp = 0.1 * max_disp + 0.8 * max_disp * _upsample_bilinear(dgrid, H, W)
    # right(x) = left(x + d(x)), linear interpolation with border clamp
    xs = np.arange(W)[None, :] + disp
    xs = np.clip(xs, 0.0, W - 1.0)
    x0 = np.floor(xs).astype(np.int64)
    x1 = np.minimum(x0 + 1, W - 1)
    wx = xs - x0
    rows = np.arange(H)[:, None]
    right = np.stack([c[rows, x0] * (1 - wx) + c[rows, x1] * wx for c in left], 0)
    mono = (disp - disp.min()) / (disp.max() - disp.min())
    return {
        "left": left.astype(np.float32),
        "right": right.astype(np.float32),
        "mono_left": mono[None].astype(np.float32),
        "mono_right": mono[None].astype(np.float32),
        "disp": disp.astype(np.float32),
    }


def synthetic_batch(B: int, H: int, W: int, max_disp: float, seed0: int = 1) -> Dict[str, np.ndarray]:
    """Stack ``B`` pairs with seeds seed0 .. seed0+B-1 into [B,C,H,W] arrays."""
    pairs = [synthetic_pair(H, W, max_disp, seed0 + i) for i in range(B)]
    return {k: np.stack([p[k] for p in pairs], 0) for k in pairs[0]}


def digest(arrays: Iterable[np.ndarray]) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def pad_to_multiple(x: np.ndarray, m: int = 32) -> Tuple[np.ndarray, Tuple[int, int, int, int]]:
    """Replicate-pad [..., H, W] up to multiples of ``m`` the way test.py:206-213 does
    (left/top get pad//2, right/bottom the rest). Returns (padded, (top, bottom, left, right))."""
    H, W = x.shape[-2:]
    ph = (m - H % m) % m
    pw = (m - W % m) % m
    t, l = ph // 2, pw // 2
    pads = [(0, 0)] * (x.ndim - 2) + [(t, ph - t), (l, pw - l)]
    return np.pad(x, pads, mode="edge"), (t, ph - t, l, pw - l)
