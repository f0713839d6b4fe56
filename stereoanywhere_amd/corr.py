"""HIP implementation of the reference's correlation plug-in point.

Reference contract (models/stereoanywhere/corr.py):
  * ``CorrBlock1D.corr(fmap2 [B,C,H,W1], fmap3 [B,C,H,W2]) -> [B,H,W1,1,W2]`` (117-132)
  * ``CorrBlock1D(fullcorr, num_levels=4, radius=4, pad=[0,0])`` builds the pyramid (76-91)
  * ``block(coords [B,2,H,W]) -> [B, num_levels*(2r+1), H, W - pad0 - pad1]`` (93-115)
selected by ``args.corr_implementation`` (stereoanywhere.py:25, 128-133).

``HipCorrBlock1D`` keeps that contract; the pyramid lives in one buffer with the levels
of a pixel row back to back (include/stereoanywhere_hip.h) and ``corr_pyramid`` exposes
per-level views shaped like the reference's.  ``HipCorrBlock1D.from_features`` is the
fused entry (volume + truncation + pyramid in one kernel) the model uses.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import ops


class HipCorrBlock1D:
    def __init__(self, fullcorr: Optional[torch.Tensor], num_levels: int = 4, radius: int = 4,
                 pad: Sequence[int] = (0, 0), _pyramid: Optional[torch.Tensor] = None,
                 _shape: Optional[tuple] = None):
        self.num_levels = num_levels
        self.radius = radius
        self.pad = list(pad)
        if _pyramid is None and fullcorr is None:
            if _shape is None:
                raise RuntimeError("HipCorrBlock1D needs a volume, a pyramid or (sheared-only) a shape")
        elif _pyramid is None:
            if fullcorr.dim() != 5 or fullcorr.shape[3] != 1:
                raise RuntimeError(f"fullcorr must be [B,H,W1,1,W2], got {tuple(fullcorr.shape)}")
            B, H, W1, _, W2 = fullcorr.shape
            _pyramid = ops.pyramid_from_volume(fullcorr.reshape(B * H * W1, W2), num_levels)
            _shape = (B, H, W1, W2)
        self.shape = _shape
        self.pyramid = _pyramid
        self.sheared = None   # disparity-sheared copy for the fused lookup (shear())
        self._views = None

    @property
    def corr_pyramid(self):
        """The reference's ``corr_pyramid`` list (corr.py:85-91): num_levels + 1 tensors of
        shape [B*H*W1, 1, 1, W2 >> i].  Levels 0..num_levels-1 are views of the lookup's
        buffer; the last level, which the reference builds and never reads, is pooled from
        the one before it on first access (one HIP pyramid launch), not in the forward."""
        if self._views is None:
            B, H, W1, W2 = self.shape
            _, offs, wids = ops.pyramid_geometry(W2, self.num_levels)
            views = [self.pyramid[:, o:o + w].unsqueeze(1).unsqueeze(1) for o, w in zip(offs, wids)]
            last = views[-1].reshape(-1, wids[-1])
            if wids[-1] >= 2:
                extra = ops.pyramid_from_volume(last.contiguous(), 2)
                w = wids[-1] // 2
                views.append(extra[:, wids[-1]:wids[-1] + w].unsqueeze(1).unsqueeze(1))
            else:   # avg_pool2d of a width-1 (or 0) row is empty
                views.append(last.new_empty((last.shape[0], 1, 1, 0)))
            self._views = views
        return self._views

    @classmethod
    def from_features(cls, fmap2: torch.Tensor, fmap3: torch.Tensor, num_levels: int = 4, radius: int = 4,
                      trunc_disp: Optional[torch.Tensor] = None, trunc_conf: Optional[torch.Tensor] = None,
                      attenuation: float = 0.9, pad: Sequence[int] = (0, 0),
                      sheared: bool = False) -> "HipCorrBlock1D":
        """corr -> x truncation volume -> pyramid fused (stereoanywhere.py:135, 201-205, 253-255).
        sheared: write the disparity-sheared layout only (ops.corr_volume_pyramid_sheared; the
        row layout where that kernel does not apply)."""
        B, _, H, W1 = fmap2.shape
        W2 = fmap3.shape[3]
        if sheared:
            sh = ops.corr_volume_pyramid_sheared(fmap2, fmap3, num_levels, trunc_disp, trunc_conf, attenuation)
            if sh is not None:
                blk = cls(None, num_levels, radius, pad, _shape=(B, H, W1, W2))
                blk.sheared = sh
                return blk
        pyr = ops.corr_volume_pyramid(fmap2, fmap3, num_levels, trunc_disp, trunc_conf, attenuation)
        return cls(None, num_levels, radius, pad, _pyramid=pyr, _shape=(B, H, W1, W2))

    def lookup_into(self, coords_x: torch.Tensor, out: torch.Tensor, other: Optional["HipCorrBlock1D"] = None):
        """Look up this pyramid (and ``other``'s, same geometry) at coords_x [B,1,H,W1] into
        out [B, nvol*L*(2r+1), H, W1] — one launch for both volumes."""
        ops.corr_lookup(self.pyramid, None if other is None else other.pyramid, self.shape[3], self.num_levels,
                        self.radius, coords_x, out)
        return out

    def shear(self, release: bool = False) -> "HipCorrBlock1D":
        """Build the disparity-sheared copy the fused lookup reads (ops.corr_pyramid_shear);
        release: drop the row-layout buffer afterwards (the per-level views need it)."""
        B, H, W1, W2 = self.shape
        self.sheared = ops.corr_pyramid_shear(self.pyramid, B, H, W1, W2, self.num_levels)
        if release:
            self.pyramid, self._views = None, None
        return self

    def lookup_conv1x1_into(self, coords_x: torch.Tensor, weight_kc: torch.Tensor, bias: torch.Tensor,
                            out: torch.Tensor, other: Optional["HipCorrBlock1D"] = None):
        """Lookup of this pyramid (and ``other``'s) followed, in the same kernel, by a 1x1 conv
        + bias + ReLU of the taps -> out [B*nvol, Cout, H, W1] (sample b*nvol + v); on the
        sheared copies when both blocks have one."""
        if self.sheared is not None and (other is None or other.sheared is not None):
            return ops.corr_lookup_conv1x1_sheared(self.sheared, None if other is None else other.sheared,
                                                   self.shape[3], self.num_levels, self.radius, coords_x, weight_kc,
                                                   bias, out)
        return ops.corr_lookup_conv1x1(self.pyramid, None if other is None else other.pyramid, self.shape[3],
                                       self.num_levels, self.radius, coords_x, weight_kc, bias, out)

    def __call__(self, coords: torch.Tensor) -> torch.Tensor:
        x = coords[:, :1]
        if self.pad[0]:
            x = x + self.pad[0]
        if not x.is_contiguous() and x.stride(3) != 1:
            x = x.contiguous()
        out = ops.corr_lookup(self.pyramid, None, self.shape[3], self.num_levels, self.radius, x)
        W1 = out.shape[-1]
        if self.pad[0] or self.pad[1]:
            out = out[..., self.pad[0]:W1 - self.pad[1]].contiguous()
        return out

    @staticmethod
    def corr(fmap2: torch.Tensor, fmap3: torch.Tensor) -> torch.Tensor:
        return ops.corr_volume(fmap2.float().contiguous(), fmap3.float().contiguous())


class CorrSampler(torch.autograd.Function):
    """Replacement of the reference's native-sampler hook (corr.py:17-29,
    ``corr_sampler.forward(volume [B,H,W1,W_i], coords [B,1,H,W1], radius)`` -> the 2r+1 taps
    of one pyramid level at x = coords, linear interpolation, zero outside [0, W_i - 1]).
    Forward only (the inference tier): one HIP lookup over a one-level pyramid."""

    @staticmethod
    def forward(ctx, volume, coords, radius):
        B, H, W1, Wi = volume.shape
        pyr = ops.pyramid_from_volume(volume.contiguous().reshape(B * H * W1, Wi), 1)
        return ops.corr_lookup(pyr, None, Wi, 1, int(radius), coords[:, :1].contiguous())

    @staticmethod
    def backward(ctx, grad_output):
        raise NotImplementedError("CorrSampler.backward: training is outside this tier")


# args.corr_implementation -> block class.  The reference's "reg" (torch) and "reg_cuda"
# (unvendored RAFT sampler, broken at corr.py:56) both resolve to the HIP block: this
# package IS the replacement of that plug-in point, and it has no CPU fallback.
CORR_IMPLEMENTATIONS = {"hip": HipCorrBlock1D, "reg": HipCorrBlock1D, "reg_cuda": HipCorrBlock1D}


def get_corr_block(name: str):
    try:
        return CORR_IMPLEMENTATIONS[name]
    except KeyError:
        raise NotImplementedError(f"corr_implementation={name!r}") from None
