"""Torch-tensor front end of the C ABI (include/stereoanywhere_hip.h).

Every function checks device / dtype / layout, allocates outputs with the caching
allocator on the input's device, and enqueues the HIP kernel on torch's current
stream through ``_native.call`` — there is no CPU or eager-torch fallback.
PyTorch is plumbing here (device memory, streams); the arithmetic is in the .so.
"""
from __future__ import annotations

import ctypes
import os
import math
from typing import List, Optional, Tuple

import torch

from . import _native as N


# algorithmic work per kernel family, accumulated while a dict is installed here (bench.py
# runs one untimed forward with it to price the families whose work depends on the layer mix)
WORK: Optional[dict] = None


def _account(kernel: str, amount: float) -> None:
    if WORK is not None:
        WORK[kernel] = WORK.get(kernel, 0.0) + amount


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(t: torch.Tensor, name: str, contiguous: bool = True) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} must be on the GPU (HIP path has no CPU fallback), got {t.device}")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def _plane_bs(t: torch.Tensor, name: str, planes: int = 1) -> int:
    """Batch stride of a [B, C, H, W] (possibly channel-sliced) view whose first
    ``planes`` channels are each dense [H, W] planes laid out back to back."""
    _check(t, name, contiguous=False)
    B, C, H, W = t.shape
    if t.stride(3) != 1 or t.stride(2) != W or (C > 1 and t.stride(1) != H * W):
        raise RuntimeError(f"{name}: inner [C,H,W] block must be dense (strides {t.stride()})")
    return t.stride(0)


# ----------------------------------------------------------------------- pyramid geometry
def pyramid_geometry(w2: int, num_levels: int) -> Tuple[int, List[int], List[int]]:
    lib = N.lib()
    rs = lib.sa_pyramid_row_stride(w2, num_levels)
    offs = [lib.sa_pyramid_level_offset(w2, i) for i in range(num_levels)]
    wids = [lib.sa_pyramid_level_width(w2, i) for i in range(num_levels)]
    return int(rs), offs, wids


# ----------------------------------------------------------------------- a1 + a8 + a9
def corr_volume_pyramid(fmap2: torch.Tensor, fmap3: torch.Tensor, num_levels: int = 4,
                        trunc_disp: Optional[torch.Tensor] = None, trunc_conf: Optional[torch.Tensor] = None,
                        attenuation: float = 0.9, row_stride: Optional[int] = None) -> torch.Tensor:
    """Stereo correlation volume (corr.py:117-132), optionally x truncation volume
    (utils.py:216-238), and its avg-pool pyramid (corr.py:76-91) in one kernel.
    Returns the pyramid buffer [B*H*W1, row_stride]."""
    _check(fmap2, "fmap2")
    _check(fmap3, "fmap3")
    B, C, H, W1 = fmap2.shape
    B3, C3, H3, W2 = fmap3.shape
    if (B3, C3, H3) != (B, C, H):
        raise RuntimeError(f"fmap shapes disagree: {tuple(fmap2.shape)} vs {tuple(fmap3.shape)}")
    if trunc_disp is not None:
        _check(trunc_disp, "trunc_disp")
        _check(trunc_conf, "trunc_conf")
        if trunc_disp.numel() != B * H * W1 or trunc_conf.numel() != B * H * W1:
            raise RuntimeError("truncation maps must be [B,1,H,W1]")
    rs = row_stride if row_stride is not None else pyramid_geometry(W2, num_levels)[0]
    out = torch.empty((B * H * W1, rs), device=fmap2.device, dtype=torch.float32)
    # torch.sqrt(torch.tensor(C)) of the reference: a float32 square root
    sqrt_c = float(torch.sqrt(torch.tensor(float(C), dtype=torch.float32)))
    N.call("sa_corr_volume_pyramid", fmap2.data_ptr(), fmap3.data_ptr(), B, C, H, W1, W2, sqrt_c,
           _ptr(trunc_disp), _ptr(trunc_conf), attenuation, num_levels, out.data_ptr(), rs, _stream(fmap2))
    return out


def corr_volume_pyramid_sheared(fmap2: torch.Tensor, fmap3: torch.Tensor, num_levels: int = 4,
                                trunc_disp: Optional[torch.Tensor] = None, trunc_conf: Optional[torch.Tensor] = None,
                                attenuation: float = 0.9) -> Optional[torch.Tensor]:
    """corr_volume_pyramid written straight in the disparity-sheared layout [B*H, slice] that
    corr_lookup_conv1x1_sheared reads (sa_corr_volume_pyramid_sheared: the same cells as
    corr_pyramid_shear(corr_volume_pyramid(...))); None where the kernel's preconditions fail
    (C % 16, W1 % 4, W2 % 4, 16-byte aligned feature maps under 2 GiB)."""
    _check(fmap2, "fmap2")
    _check(fmap3, "fmap3")
    B, C, H, W1 = fmap2.shape
    W2 = fmap3.shape[3]
    if tuple(fmap3.shape[:3]) != (B, C, H):
        raise RuntimeError(f"fmap shapes disagree: {tuple(fmap2.shape)} vs {tuple(fmap3.shape)}")
    lim = (1 << 31) - 64
    if (C % 16 or W1 % 4 or W2 % 4 or fmap2.data_ptr() % 16 or fmap3.data_ptr() % 16
            or fmap2.numel() * 4 >= lim or fmap3.numel() * 4 >= lim):
        return None
    if trunc_disp is not None:
        _check(trunc_disp, "trunc_disp")
        _check(trunc_conf, "trunc_conf")
        if trunc_disp.numel() != B * H * W1 or trunc_conf.numel() != B * H * W1:
            raise RuntimeError("truncation maps must be [B,1,H,W1]")
    slice_sz = int(N.lib().sa_shear_slice_size(W1, W2, num_levels))
    out = torch.empty((B * H, slice_sz), device=fmap2.device, dtype=torch.float32)
    sqrt_c = float(torch.sqrt(torch.tensor(float(C), dtype=torch.float32)))
    N.call("sa_corr_volume_pyramid_sheared", fmap2.data_ptr(), fmap3.data_ptr(), B, C, H, W1, W2, sqrt_c,
           _ptr(trunc_disp), _ptr(trunc_conf), attenuation, num_levels, out.data_ptr(), _stream(fmap2))
    return out


def pyramid_from_volume_sheared(volume: torch.Tensor, num_levels: int = 4) -> Optional[torch.Tensor]:
    """pyramid_from_volume of a [B, 1, H, W1, W2] view of a [B, 1, W2, H, W1] volume (the
    hourglass classifier's layout) written in the disparity-sheared layout [B*H, slice]
    (sa_corr_pyramid_from_volume_strided_sheared); None for any other layout."""
    _check(volume, "volume", contiguous=False)
    if not (volume.dim() == 5 and volume.shape[1] == 1 and volume.stride(-1) != 1 and volume.stride(3) == 1
            and volume.shape[3] % 4 == 0 and volume.data_ptr() % 16 == 0
            and all(volume.stride(i) % 4 == 0 for i in (0, 2, 4))):
        return None
    B, _, H, W1, W2 = volume.shape
    slice_sz = int(N.lib().sa_shear_slice_size(W1, W2, num_levels))
    out = torch.empty((B * H, slice_sz), device=volume.device, dtype=torch.float32)
    N.call("sa_corr_pyramid_from_volume_strided_sheared", volume.data_ptr(), B, H, W1, W2, volume.stride(0),
           volume.stride(2), volume.stride(4), num_levels, out.data_ptr(), _stream(volume))
    _account("mono_pyramid", 4.0 * B * H * W1 * (W2 + sum(pyramid_geometry(W2, num_levels)[2])))
    return out


def corr_volume(fmap2: torch.Tensor, fmap3: torch.Tensor) -> torch.Tensor:
    """CorrBlock1D.corr contract: [B,C,H,W1] x [B,C,H,W2] -> [B,H,W1,1,W2]."""
    B, C, H, W1 = fmap2.shape
    W2 = fmap3.shape[3]
    vol = corr_volume_pyramid(fmap2, fmap3, num_levels=1, row_stride=W2)
    return vol.view(B, H, W1, 1, W2)


def pyramid_from_volume(volume: torch.Tensor, num_levels: int = 4) -> torch.Tensor:
    """CorrBlock1D.__init__ on an existing volume [..., W2] (rows contiguous along W2), or on a
    [B, 1, H, W1, W2] view whose W1 axis is the contiguous one (any W2; needs W1 % 4 == 0 and
    16-byte aligned rows, else the view is made contiguous first)."""
    _check(volume, "volume", contiguous=False)
    W2 = volume.shape[-1]
    if (volume.dim() == 5 and volume.shape[1] == 1 and volume.stride(-1) != 1 and volume.stride(3) == 1
            and volume.shape[3] % 4 == 0 and volume.data_ptr() % 16 == 0
            and all(volume.stride(i) % 4 == 0 for i in (0, 2, 4))):
        # [B, 1, H, W1, W2] view of a [B, 1, W2, H, W1] volume: transposed while staging
        B, _, H, W1, _ = volume.shape
        rs = pyramid_geometry(W2, num_levels)[0]
        out = torch.empty((B * H * W1, rs), device=volume.device, dtype=torch.float32)
        N.call("sa_corr_pyramid_from_volume_strided", volume.data_ptr(), B, H, W1, W2, volume.stride(0),
               volume.stride(2), volume.stride(4), num_levels, out.data_ptr(), rs, _stream(volume))
        # the volume read once, every level cell written once
        _account("mono_pyramid", 4.0 * B * H * W1 * (W2 + sum(pyramid_geometry(W2, num_levels)[2])))
        return out
    rows2d = volume.reshape(-1, W2)
    if rows2d.stride(1) != 1 and volume.dim() == 5:   # a strided view the kernel above cannot take
        rows2d = volume.contiguous().reshape(-1, W2)
    if rows2d.stride(1) != 1:
        raise RuntimeError("volume rows must be contiguous along the last axis")
    rs = pyramid_geometry(W2, num_levels)[0]
    out = torch.empty((rows2d.shape[0], rs), device=volume.device, dtype=torch.float32)
    N.call("sa_corr_pyramid_from_volume", rows2d.data_ptr(), rows2d.shape[0], W2, rows2d.stride(0),
           num_levels, out.data_ptr(), rs, _stream(volume))
    _account("mono_pyramid", 4.0 * rows2d.shape[0] * (W2 + sum(pyramid_geometry(W2, num_levels)[2])))
    return out


# ----------------------------------------------------------------------- a10
def corr_lookup(pyr_a: torch.Tensor, pyr_b: Optional[torch.Tensor], W2: int, num_levels: int, radius: int,
                coords_x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Lookup of one or two pyramids at coords_x [B,1,H,W1] (any batch stride) ->
    out [B, nvol*L*(2r+1), H, W1] (stereo channels first, then mono)."""
    _check(pyr_a, "pyramid_a")
    if pyr_b is not None:
        _check(pyr_b, "pyramid_b")
        if pyr_b.shape != pyr_a.shape:
            raise RuntimeError("both pyramids must share a geometry")
    cbs = _plane_bs(coords_x, "coords_x")
    B, _, H, W1 = coords_x.shape
    rs = pyr_a.shape[1]
    if pyr_a.shape[0] != B * H * W1:
        raise RuntimeError(f"pyramid rows {pyr_a.shape[0]} != B*H*W1 {B * H * W1}")
    nvol = 2 if pyr_b is not None else 1
    K = 2 * radius + 1
    if out is None:
        out = torch.empty((B, nvol * num_levels * K, H, W1), device=pyr_a.device, dtype=torch.float32)
    obs = _plane_bs(out, "out")
    N.call("sa_corr_lookup", pyr_a.data_ptr(), _ptr(pyr_b), W2, rs, num_levels, radius, coords_x.data_ptr(),
           cbs, B, H, W1, out.data_ptr(), obs, _stream(pyr_a))
    return out


def corr_lookup_conv1x1(pyr_a: torch.Tensor, pyr_b: Optional[torch.Tensor], W2: int, num_levels: int, radius: int,
                        coords_x: torch.Tensor, weight_kc: torch.Tensor, bias: torch.Tensor,
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Lookup fused with a 1x1 conv + bias + ReLU of the taps (the motion encoder's convc1):
    weight_kc [L*(2r+1), Cout] -> out [B*nvol, Cout, H, W1], sample b*nvol + v."""
    _check(pyr_a, "pyramid_a")
    if pyr_b is not None:
        _check(pyr_b, "pyramid_b")
        if pyr_b.shape != pyr_a.shape:
            raise RuntimeError("both pyramids must share a geometry")
    _check(weight_kc, "weight_kc")
    _check(bias, "bias")
    cbs = _plane_bs(coords_x, "coords_x")
    B, _, H, W1 = coords_x.shape
    if pyr_a.shape[0] != B * H * W1:
        raise RuntimeError(f"pyramid rows {pyr_a.shape[0]} != B*H*W1 {B * H * W1}")
    nvol = 2 if pyr_b is not None else 1
    Cout = weight_kc.shape[1]
    if weight_kc.shape[0] != num_levels * (2 * radius + 1):
        raise RuntimeError("weight_kc must be [L*(2r+1), Cout]")
    if out is None:
        out = torch.empty((B * nvol, Cout, H, W1), device=pyr_a.device, dtype=torch.float32)
    _check(out, "out")
    N.call("sa_corr_lookup_conv1x1", pyr_a.data_ptr(), _ptr(pyr_b), W2, pyr_a.shape[1], num_levels, radius,
           coords_x.data_ptr(), cbs, B, H, W1, weight_kc.data_ptr(), bias.data_ptr(), Cout, out.data_ptr(),
           _stream(pyr_a))
    return out


def shear_supported(B: int, H: int, W1: int, W2: int, num_levels: int = 4) -> bool:
    """Whether the sheared lookup pipeline takes this geometry (sa_corr_shear_supported: B*H <=
    65535 image rows, W2 <= 511 for the shear pass's LDS tile, 4 levels); else the row layout."""
    return bool(N.lib().sa_corr_shear_supported(B, H, W1, W2, num_levels))


def corr_pyramid_shear(pyr: torch.Tensor, B: int, H: int, W1: int, W2: int, num_levels: int = 4) -> torch.Tensor:
    """Row-layout pyramid [B*H*W1, row_stride] -> its disparity-sheared copy [B*H, slice]
    (sa_corr_pyramid_shear; read by corr_lookup_conv1x1_sheared)."""
    _check(pyr, "pyramid")
    if pyr.shape[0] != B * H * W1:
        raise RuntimeError(f"pyramid rows {pyr.shape[0]} != B*H*W1 {B * H * W1}")
    slice_sz = int(N.lib().sa_shear_slice_size(W1, W2, num_levels))
    out = torch.empty((B * H, slice_sz), device=pyr.device, dtype=torch.float32)
    N.call("sa_corr_pyramid_shear", pyr.data_ptr(), pyr.shape[1], B, H, W1, W2, num_levels, out.data_ptr(),
           _stream(pyr))
    return out


def corr_lookup_conv1x1_sheared(sh_a: torch.Tensor, sh_b: Optional[torch.Tensor], W2: int, num_levels: int,
                                radius: int, coords_x: torch.Tensor, weight_kc: torch.Tensor, bias: torch.Tensor,
                                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """corr_lookup_conv1x1 on sheared pyramids [B*H, slice] (corr_pyramid_shear)."""
    _check(sh_a, "sheared_a")
    if sh_b is not None:
        _check(sh_b, "sheared_b")
        if sh_b.shape != sh_a.shape:
            raise RuntimeError("both sheared pyramids must share a geometry")
    _check(weight_kc, "weight_kc")
    _check(bias, "bias")
    cbs = _plane_bs(coords_x, "coords_x")
    B, _, H, W1 = coords_x.shape
    if sh_a.shape != (B * H, int(N.lib().sa_shear_slice_size(W1, W2, num_levels))):
        raise RuntimeError(f"sheared pyramid {tuple(sh_a.shape)} does not match coords {tuple(coords_x.shape)}")
    nvol = 2 if sh_b is not None else 1
    Cout = weight_kc.shape[1]
    if out is None:
        out = torch.empty((B * nvol, Cout, H, W1), device=sh_a.device, dtype=torch.float32)
    _check(out, "out")
    N.call("sa_corr_lookup_conv1x1_sheared", sh_a.data_ptr(), _ptr(sh_b), W2, num_levels, radius,
           coords_x.data_ptr(), cbs, B, H, W1, weight_kc.data_ptr(), bias.data_ptr(), Cout, out.data_ptr(),
           _stream(sh_a))
    return out


# ----------------------------------------------------------------------- a2 + a3
def mono_normals(mde_lowres: torch.Tensor, gain: float) -> torch.Tensor:
    _check(mde_lowres, "mde_lowres")
    B, _, H, W = mde_lowres.shape
    out = torch.empty((B, 3, H, W), device=mde_lowres.device, dtype=torch.float32)
    N.call("sa_mono_normals", mde_lowres.data_ptr(), B, H, W, gain, out.data_ptr(), _stream(mde_lowres))
    return out


def mono_masked_volume(n2, n3, m2, m3, nbins: int = 8, gain: float = 1.73) -> torch.Tensor:
    """-> [B, nbins, W2, H, W1] (the hourglass's working layout)."""
    for t, nm in ((n2, "n2"), (n3, "n3"), (m2, "m2"), (m3, "m3")):
        _check(t, nm)
    B, _, H, W1 = n2.shape
    W2 = n3.shape[3]
    out = torch.empty((B, nbins, W2, H, W1), device=n2.device, dtype=torch.float32)
    N.call("sa_mono_masked_volume", n2.data_ptr(), n3.data_ptr(), m2.data_ptr(), m3.data_ptr(), B, H, W1, W2,
           nbins, gain, out.data_ptr(), _stream(n2))
    return out


def mono_bin_records(normals: torch.Tensor, m: torch.Tensor, nbins: int = 8) -> torch.Tensor:
    """-> [B, H, W, 4] records (n0, n1, n2, depth bin or -1) of one view (sa_mono_bin_records)."""
    _check(normals, "normals")
    _check(m, "m")
    B, _, H, W = normals.shape
    rec = torch.empty((B, H, W, 4), device=normals.device, dtype=torch.float32)
    N.call("sa_mono_bin_records", normals.data_ptr(), m.data_ptr(), B, H, W, nbins, rec.data_ptr(), _stream(rec))
    return rec


class OneHotVolume:
    """The masked mono volume [B, nbins, W2, H, W1] (stereoanywhere.py:161) by its per-pixel
    records: cell (n, k, h, j) = gain * nL[h,j] . nR[h,k] / sqrt(3) iff both pixels are in bin n.
    The fused hourglass's readers of the volume (ops.conv3d at stride 2, ops.conv3d_pointwise_upcat)
    evaluate the cells from the records; nothing of the volume is written."""

    def __init__(self, n2, n3, m2, m3, nbins: int = 8, gain: float = 1.73):
        self.rec_l, self.rec_r = mono_bin_records(n2, m2, nbins), mono_bin_records(n3, m3, nbins)
        self.nbins, self.gain = nbins, gain
        B, _, H, W1 = n2.shape
        self.shape = torch.Size((B, nbins, n3.shape[3], H, W1))
        self.device = n2.device


# ----------------------------------------------------------------------- a5 + a6
def softargmin_conf(vol_disp: Optional[torch.Tensor], vol_conf: Optional[torch.Tensor], strides, dims,
                    out_disp: Optional[torch.Tensor] = None, out_conf: Optional[torch.Tensor] = None):
    """Volumes addressed as v[b*sb + h*sh + j*sj + k*sk] with dims (B, H, W1, W2).
    Outputs are [B, 2, H, W] buffers: channel 0 = left (over k), 1 = right (over j)."""
    B, H, W1, W2 = dims
    if W1 != W2:
        raise RuntimeError("joint [B,2,H,W] outputs need W1 == W2")
    sb, sh, sj, sk = strides
    ref = vol_disp if vol_disp is not None else vol_conf
    if out_disp is None and vol_disp is not None:
        out_disp = torch.empty((B, 2, H, W1), device=ref.device, dtype=torch.float32)
    if out_conf is None and vol_conf is not None:
        out_conf = torch.empty((B, 2, H, W1), device=ref.device, dtype=torch.float32)
    obs = 2 * H * W1
    dL = dR = cL = cR = None
    if out_disp is not None:
        dL, dR = out_disp.data_ptr(), out_disp[:, 1].data_ptr()
    if out_conf is not None:
        cL, cR = out_conf.data_ptr(), out_conf[:, 1].data_ptr()
    N.call("sa_softargmin_conf", _ptr(vol_disp), _ptr(vol_conf), B, H, W1, W2, sb, sh, sj, sk, dL, dR, cL, cR,
           obs, _stream(ref))
    return out_disp, out_conf


# ----------------------------------------------------------------------- a7 + a8 + a11
def softlrc_joint(disp: torch.Tensor, conf: Optional[torch.Tensor], lrc_th: float) -> torch.Tensor:
    """softlrc of the L/R halves of a [B,2,H,W] disparity buffer, times conf (fuzzy_and)
    when given -> [B,2,H,W]."""
    _check(disp, "disp")
    B, _, H, W = disp.shape
    out = torch.empty_like(disp)
    c2 = c3 = None
    if conf is not None:
        _check(conf, "conf")
        c2, c3 = conf.data_ptr(), conf[:, 1].data_ptr()
    N.call("sa_softlrc", disp.data_ptr(), disp[:, 1].data_ptr(), c2, c3, B, H, W, 2 * H * W, lrc_th,
           out.data_ptr(), out[:, 1].data_ptr(), _stream(disp))
    return out


def weighted_lsq(mde: torch.Tensor, disp: torch.Tensor, conf: torch.Tensor, q_lo: float = 0.2,
                 q_hi: float = 0.9, single_block: Optional[bool] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-sample (scale, shift) [B] of weighted_lsq over the flattened [B, ...] maps.
    One launch, one workgroup per sample (sa_weighted_lsq, the default since round 6: B=4 at
    2x136x240 73-77 vs ~100 us for the five-launch grid form, B=64 76 vs 714 us), or spread over
    the GPU with a zeroed workspace (sa_weighted_lsq_ws, single_block=False)."""
    for t, nm in ((mde, "mde"), (disp, "disp"), (conf, "conf")):
        _check(t, nm)
    B = mde.shape[0]
    n = mde.numel() // B
    scale = torch.empty(B, device=mde.device, dtype=torch.float32)
    shift = torch.empty(B, device=mde.device, dtype=torch.float32)
    if single_block is None:
        single_block = True
    if single_block:
        N.call("sa_weighted_lsq", mde.data_ptr(), disp.data_ptr(), conf.data_ptr(), B, n, q_lo, q_hi,
               scale.data_ptr(), shift.data_ptr(), _stream(mde))
    else:
        ws = torch.zeros(int(N.lib().sa_weighted_lsq_ws_size(B, n)), device=mde.device, dtype=torch.uint8)
        N.call("sa_weighted_lsq_ws", mde.data_ptr(), disp.data_ptr(), conf.data_ptr(), B, n, q_lo, q_hi,
               scale.data_ptr(), shift.data_ptr(), ws.data_ptr(), _stream(mde))
    return scale, shift


def mono_scale_mirror(mde_lr: torch.Tensor, scale, shift, disp: torch.Tensor, conf: torch.Tensor, lrc_th: float,
                      conf_th: float):
    """From [B,2,H,W] mono / disparity / confidence buffers -> sm2, sm3, mirror, coords_x [B,1,H,W]."""
    for t, nm in ((mde_lr, "mde_lr"), (disp, "disp"), (conf, "conf")):
        _check(t, nm)
    B, _, H, W = mde_lr.shape
    outs = [torch.empty((B, 1, H, W), device=mde_lr.device, dtype=torch.float32) for _ in range(4)]
    N.call("sa_mono_scale_mirror", mde_lr.data_ptr(), mde_lr[:, 1].data_ptr(), scale.data_ptr(), shift.data_ptr(),
           disp.data_ptr(), conf.data_ptr(), B, H, W, 2 * H * W, lrc_th, conf_th,
           *[o.data_ptr() for o in outs], _stream(mde_lr))
    return tuple(outs)


# ----------------------------------------------------------------------- a12 / a13 plumbing
def gru_zr(xc, hzr, cz, cr, h, z_out, rh_out, bx: Optional[torch.Tensor] = None):
    """z = sigmoid(xc_z + bx_z + hzr_z + cz), r*h with r = sigmoid(xc_r + bx_r + hzr_r + cr)."""
    B, C, H, W = h.shape
    N.call("sa_gru_zr", xc.data_ptr(), _plane_bs(xc, "xc"), _ptr(bx), hzr.data_ptr(), _plane_bs(hzr, "hzr"),
           cz.data_ptr(), cr.data_ptr(), _plane_bs(cz, "cz"), h.data_ptr(), _plane_bs(h, "h"), B, C, H * W,
           z_out.data_ptr(), rh_out.data_ptr(), _stream(h))
    # xc (z, r), hzr (z, r), cz, cr, h read; z, r*h written
    _account("gru_zr", 4.0 * 9 * B * C * H * W)


def gru_out(xc, qh, cq, z, h, bx: Optional[torch.Tensor] = None, qh2: Optional[torch.Tensor] = None):
    """h = (1 - z) h + z tanh(xc_q + bx_q + qh (+ qh2) + cq), in place; qh2: the second partial sum
    of an r*h conv split over its input channels (same layout as qh)."""
    B, C, H, W = h.shape
    if qh2 is not None and (qh2.shape != qh.shape or _plane_bs(qh2, "qh2") != _plane_bs(qh, "qh")):
        raise RuntimeError("gru_out: qh2 must match qh's shape and batch stride")
    N.call("sa_gru_out_split", xc.data_ptr(), _plane_bs(xc, "xc"), _ptr(bx), qh.data_ptr(), _ptr(qh2),
           _plane_bs(qh, "qh"), cq.data_ptr(), _plane_bs(cq, "cq"), z.data_ptr(), B, C, H * W, h.data_ptr(),
           _plane_bs(h, "h"), _stream(h))
    # xc_q, qh (+ qh2), cq, z, h read; h written
    _account("gru_out", 4.0 * (6 + (qh2 is not None)) * B * C * H * W)


def _pitched_bs(t: torch.Tensor, name: str) -> int:
    """Batch stride of a [B, C, H, P] (possibly channel-sliced) view of dense [H, P] planes."""
    _check(t, name, contiguous=False)
    B, C, H, P = t.shape
    if t.stride(3) != 1 or t.stride(2) != P or (C > 1 and t.stride(1) != H * P):
        raise RuntimeError(f"{name}: inner [C,H,P] block must be dense (strides {t.stride()})")
    return t.stride(0)


def pool2x(x: torch.Tensor, out: torch.Tensor, width: Optional[int] = None,
           out_width: Optional[int] = None) -> torch.Tensor:
    """avg_pool2d(3, 2, 1) of x [B,C,H,W] into out [B,C,Ho,Wo]; width / out_width: the image
    widths of pitched planes (the last dimension is then the row pitch; pad columns untouched)."""
    B, C, H, Px = x.shape
    W = width or Px
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    Po = out.shape[3]
    if (out_width or Po) != Wo or tuple(out.shape[:3]) != (B, C, Ho):
        raise RuntimeError(f"pool2x: out {tuple(out.shape)} (width {out_width}) != {(B, C, Ho, Wo)}")
    N.call("sa_pool2x_p", x.data_ptr(), _pitched_bs(x, "x"), Px, B, C, H, W, out.data_ptr(),
           _pitched_bs(out, "out"), Po, _stream(x))
    _account("gru_plumbing", 4.0 * B * C * (H * W + Ho * Wo))   # input read once, output written
    return out


def interp(x: torch.Tensor, out: torch.Tensor, width: Optional[int] = None,
           out_width: Optional[int] = None) -> torch.Tensor:
    """Bilinear align_corners resize of x into out's size; width / out_width as in pool2x."""
    B, C, H, Px = x.shape
    Bo, Co, Ho, Po = out.shape
    if (Bo, Co) != (B, C):
        raise RuntimeError("interp: batch/channels mismatch")
    N.call("sa_interp_bilinear_ac_p", x.data_ptr(), _pitched_bs(x, "x"), Px, B, C, H, width or Px, Ho,
           out_width or Po, out.data_ptr(), _pitched_bs(out, "out"), Po, _stream(x))
    _account("gru_plumbing", 4.0 * B * C * (H * (width or Px) + Ho * (out_width or Po)))
    return out


_RESAMPLE_MULTI_MAX = 1 << 26   # output elements (views count their own extent)


def resample_multi(*jobs) -> None:
    """Independent pool2x / interp jobs in one launch (sa_resample_multi): each job is
    ("pool" | "interp", x, out, width, out_width) with the arguments of pool2x / interp, or
    ("flow_x", coords_x, flow_planes, None, None) = flow_update(coords_x, None, None, flow_planes)."""
    if not 1 <= len(jobs) <= 4:
        raise RuntimeError("resample_multi: 1..4 jobs")
    bad = [j[0] for j in jobs if j[0] not in ("pool", "interp", "flow_x")]
    if bad:
        raise RuntimeError(f"resample_multi: unknown job kind {bad[0]!r}")
    if sum(out.numel() for _, _, out, _, _ in jobs) > _RESAMPLE_MULTI_MAX:
        # big jobs fill the chip on their own: one launch each (the booster batch's pair took
        # 291 / 293 us merged against 274 / 274 us as two launches; configs[1]'s 19.7 / 22.4 us
        # against 28.7 / 29.0, scripts/bench_small.py --plumbing)
        for kind, x, out, width, out_width in jobs:
            if kind == "flow_x":
                flow_update(x, None, None, out)
            else:
                (pool2x if kind == "pool" else interp)(x, out, width=width, out_width=out_width)
        return
    arr = (N.SaResampleJob * len(jobs))()
    nbytes = 0.0
    for j, (kind, x, out, width, out_width) in zip(arr, jobs):
        if kind == "flow_x":   # flow_update(coords_x, None, None, out) as a job
            _check(x, "coords_x")
            B, _, H, W = x.shape
            if x.shape[1] != 1 or tuple(out.shape) != (B, 2, H, W):
                raise RuntimeError(f"resample_multi: flow job coords {tuple(x.shape)} / planes {tuple(out.shape)}")
            j.kind, j.in_, j.in_bs, j.in_pitch = 2, x.data_ptr(), x.stride(0), W
            j.B, j.C, j.H, j.W, j.Ho, j.Wo = B, 1, H, W, H, W
            j.out, j.out_bs, j.out_pitch = out.data_ptr(), _plane_bs(out, "flow_b"), W
            nbytes += 12.0 * B * H * W
            continue
        B, C, H, Px = x.shape
        W = width or Px
        Bo, Co, Ho, Po = out.shape
        Wo = out_width or Po
        if (Bo, Co) != (B, C):
            raise RuntimeError(f"resample_multi: {kind} batch/channels mismatch")
        if kind == "pool":
            if (Ho, Wo) != ((H - 1) // 2 + 1, (W - 1) // 2 + 1):
                raise RuntimeError(f"resample_multi: pool out {tuple(out.shape)} (width {out_width}) != "
                                   f"{(B, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1)}")
        if x.device != out.device:
            raise RuntimeError("resample_multi: x and out on different devices")
        j.kind = 0 if kind == "pool" else 1
        j.in_, j.in_bs, j.in_pitch = x.data_ptr(), _pitched_bs(x, "x"), Px
        j.B, j.C, j.H, j.W, j.Ho, j.Wo = B, C, H, W, Ho, Wo
        j.out, j.out_bs, j.out_pitch = out.data_ptr(), _pitched_bs(out, "out"), Po
        nbytes += 4.0 * B * C * (H * W + Ho * Wo)
    N.call("sa_resample_multi", len(jobs), ctypes.addressof(arr), _stream(jobs[0][1]))
    _account("gru_plumbing", nbytes)


def feature_gate_weights(branch) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """(w3 [32, 9], w1 [C, 32], b1 [C]) of a DoubleFeatureAtt branch (BasicConv(1 -> 32, 3x3) +
    Conv2d(32 -> C, 1x1)) for sa_feature_gates."""
    conv, lin = branch[0].conv, branch[1]
    if conv.weight.shape[1:] != (1, 3, 3) or conv.weight.shape[0] != 32 or lin.weight.shape[1:] != (32, 1, 1):
        raise RuntimeError(f"feature_gate_weights: unsupported branch {tuple(conv.weight.shape)} / "
                           f"{tuple(lin.weight.shape)}")
    b1 = None if lin.bias is None else lin.bias.detach().float().contiguous()
    return (conv.weight.detach().float().reshape(32, 9).contiguous(),
            lin.weight.detach().float().reshape(lin.weight.shape[0], 32).contiguous(), b1)


def feature_gates(jobs) -> list:
    """The DoubleFeatureAtt branch outputs sigmoid(conv1x1(leaky(IN(conv3x3(feat))))) for up to 8
    jobs (feat [B, 1, H, W], (w3, w1, b1) from feature_gate_weights) in two launches
    (sa_feature_gates); returns a [B, C, H, W] tensor per job."""
    if not 1 <= len(jobs) <= 8:
        raise RuntimeError("feature_gates: 1..8 jobs")
    arr = (N.SaFeatureGateJob * len(jobs))()
    outs = []
    nbytes = 0.0
    for j, (x, (w3, w1, b1)) in zip(arr, jobs):
        _check(x, "feat")
        B, Cin, H, W = x.shape
        if Cin != 1:
            raise RuntimeError(f"feature_gates: one-channel features, got {tuple(x.shape)}")
        for t, nm in ((w3, "w3"), (w1, "w1")):
            _check(t, nm)
        C = w1.shape[0]
        out = torch.empty(B, C, H, W, device=x.device, dtype=torch.float32)
        j.in_, j.in_bs, j.B, j.H, j.W = x.data_ptr(), x.stride(0), B, H, W
        j.w3, j.w1, j.b1, j.C = w3.data_ptr(), w1.data_ptr(), _ptr(b1), C
        j.out, j.out_bs = out.data_ptr(), out.stride(0)
        outs.append(out)
        nbytes += 4.0 * B * H * W * (2 + C)
    ws = torch.empty(int(N.lib().sa_feature_gates_ws_size(len(jobs), ctypes.addressof(arr))), dtype=torch.uint8,
                     device=jobs[0][0].device)
    N.call("sa_feature_gates", len(jobs), ctypes.addressof(arr), ws.data_ptr(), _stream(jobs[0][0]))
    _account("misc", nbytes)
    return outs


def relu_copy(x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    B, C, H, W = x.shape
    if tuple(out.shape) != (B, C, H, W):
        raise RuntimeError("relu_copy: shape mismatch")
    N.call("sa_relu_copy", x.data_ptr(), _plane_bs(x, "x"), B, C, H * W, out.data_ptr(), _plane_bs(out, "out"),
           _stream(x))
    _account("gru_plumbing", 8.0 * B * C * H * W)
    return out


def flow_update(coords_x: torch.Tensor, delta: Optional[torch.Tensor], flow_a: Optional[torch.Tensor],
                flow_b: Optional[torch.Tensor]) -> None:
    _check(coords_x, "coords_x")
    B, _, H, W = coords_x.shape
    N.call("sa_flow_update", coords_x.data_ptr(), _ptr(delta), 0 if delta is None else _plane_bs(delta, "delta"),
           B, H, W, _ptr(flow_a), 0 if flow_a is None else _plane_bs(flow_a, "flow_a"), _ptr(flow_b),
           0 if flow_b is None else _plane_bs(flow_b, "flow_b"), _stream(coords_x))
    # coords read (+ written with a delta read), each flow plane written
    _account("gru_plumbing", 4.0 * B * H * W * (1 + (2 if delta is not None else 0)
                                                + (flow_a is not None) + (flow_b is not None)))


def convex_upsample(flow_x: torch.Tensor, mask: torch.Tensor, factor: int = 4) -> torch.Tensor:
    """flow_x [B,1,H,W] (contiguous), mask [B,9*f*f,H,W] -> [B,1,f*H,f*W]."""
    _check(flow_x, "flow_x")
    B, _, H, W = flow_x.shape
    out = torch.empty((B, 1, factor * H, factor * W), device=flow_x.device, dtype=torch.float32)
    N.call("sa_convex_upsample", flow_x.data_ptr(), mask.data_ptr(), _plane_bs(mask, "mask"), B, H, W, factor,
           out.data_ptr(), _stream(flow_x))
    return out


def float32_sqrt(x: float) -> float:
    return float(torch.sqrt(torch.tensor(float(x), dtype=torch.float32)))




# ----------------------------------------------------------------------- fused hourglass tail / convf1
def conv3d_stat_parts(cout: int, stride: int, D: int, H: int, W: int) -> int:
    return int(N.lib().sa_conv3d_stat_parts(cout, stride, D, H, W))


def instnorm_finalize(partial: torch.Tensor, bc: int, parts: int, count: int, eps: float = 1e-5):
    mean = torch.empty(bc, device=partial.device, dtype=torch.float32)
    rstd = torch.empty(bc, device=partial.device, dtype=torch.float32)
    N.call("sa_instnorm_finalize", partial.data_ptr(), bc, parts, count, eps, mean.data_ptr(), rstd.data_ptr(),
           _stream(partial))
    return mean, rstd


class VolAct:
    """A raw conv output plus the transform its consumers apply on load:
    T(x) = [gate_l * gate_r *] [lrelu(] [(x - mean) * rstd] [)]."""

    def __init__(self, raw: torch.Tensor, norm=None, act: bool = False, gate=None):
        self.raw, self.norm, self.act, self.gate = raw, norm, act, gate

    def args(self):
        mean, rstd = self.norm if self.norm is not None else (None, None)
        gl, gr = self.gate if self.gate is not None else (None, None)
        return [_ptr(mean), _ptr(rstd), 1 if self.act else 0, _ptr(gl), _ptr(gr)]

    def with_gate(self, gate) -> "VolAct":
        return VolAct(self.raw, self.norm, self.act, gate)


def vol_apply(x: "VolAct", slope: float = 0.01) -> "VolAct":
    """Materialise T(x.raw) -> VolAct(out) with the identity transform."""
    _check(x.raw, "x")
    B, C, D, H, W = x.raw.shape
    out = torch.empty_like(x.raw)
    a = x.args()
    N.call("sa_vol_apply", x.raw.data_ptr(), B, C, D, H, W, a[0], a[1], a[2], slope, a[3], a[4], out.data_ptr(),
           _stream(out))
    return VolAct(out)


def conv3d(x: "VolAct", w_t: torch.Tensor, cout: int, stride: int = 1, slope: float = 0.01, stats: bool = True):
    """3x3x3 conv (pad 1, no bias) of T(x.raw); w_t pre-arranged [Cin][27][Cout].
    Returns VolAct(out, InstanceNorm stats of out if requested, act=True)."""
    if isinstance(x, OneHotVolume):
        return _conv3d_onehot(x, w_t, cout, stride, stats)
    _check(x.raw, "x")
    _check(w_t, "w_t")
    B, Cin, D, H, W = x.raw.shape
    Do, Ho, Wo = (D - 1) // stride + 1, (H - 1) // stride + 1, (W - 1) // stride + 1
    out = torch.empty((B, cout, Do, Ho, Wo), device=x.raw.device, dtype=torch.float32)
    parts = conv3d_stat_parts(cout, stride, Do, Ho, Wo)
    partial = torch.empty((B * cout * parts * 2,), device=out.device, dtype=torch.float64) if stats else None
    a = x.args()
    N.call("sa_conv3d", x.raw.data_ptr(), B, Cin, D, H, W, stride, w_t.data_ptr(), cout, a[0], a[1], a[2], slope,
           a[3], a[4], out.data_ptr(), _ptr(partial), _stream(out))
    norm = instnorm_finalize(partial, B * cout, parts, Do * Ho * Wo) if stats else None
    return VolAct(out, norm, act=stats)


# G of Winograd F(4,3) (points 0, +-1, +-2, inf; conv2d_wino4.hip's filter transform)
_G43 = ((0.25, 0.0, 0.0), (-1.0 / 6, -1.0 / 6, -1.0 / 6), (-1.0 / 6, 1.0 / 6, -1.0 / 6),
        (1.0 / 24, 1.0 / 12, 1.0 / 6), (1.0 / 24, -1.0 / 12, 1.0 / 6), (0.0, 0.0, 1.0))


def conv3d_wd_weights(w_t: torch.Tensor) -> torch.Tensor:
    """[Cin][27][Cout] 3x3x3 kernel (ops.conv3d layout) -> [Cin][3 kh][3 kw][6][Cout], the D-taps
    transformed by G of F(4,3) in float64 and rounded once (sa_conv3d_wd)."""
    cin, _, cout = w_t.shape
    G = torch.tensor(_G43, dtype=torch.float64, device=w_t.device)
    w = w_t.to(torch.float64).reshape(cin, 3, 3, 3, cout)   # [ci][kd][kh][kw][co]
    return torch.einsum("pk,ikhwc->ihwpc", G, w).to(torch.float32).contiguous()


def conv3d_wd(x: "VolAct", w_wd: torch.Tensor, cout: int, slope: float = 0.01, stats: bool = True) -> "VolAct":
    """ops.conv3d at stride 1 for 8 input channels (-> 8 or 2), 16 -> 16 or 32 -> 32 (no gate) on the
    F(4,3)-along-D kernel; w_wd from conv3d_wd_weights.  The input must carry an InstanceNorm +
    LeakyReLU (+ gate)."""
    _check(x.raw, "x")
    _check(w_wd, "w_wd")
    B, Cin, D, H, W = x.raw.shape
    out = torch.empty((B, cout, D, H, W), device=x.raw.device, dtype=torch.float32)
    parts = int(N.lib().sa_conv3d_wd_stat_parts(cout, D, H, W))
    partial = torch.empty((B * cout * parts * 2,), device=out.device, dtype=torch.float64) if stats else None
    a = x.args()
    N.call("sa_conv3d_wd", x.raw.data_ptr(), B, Cin, D, H, W, w_wd.data_ptr(), cout, a[0], a[1], a[2], slope,
           a[3], a[4], out.data_ptr(), _ptr(partial), _stream(out))
    norm = instnorm_finalize(partial, B * cout, parts, D * H * W) if stats else None
    return VolAct(out, norm, act=stats)


# the stride-1 hourglass convs 8 -> 8 and 16 -> 16 on the split-f16 MFMA kernel (conv3d_mfma.hip)
# instead of the F(4,3)-along-D VALU kernel (conv3d_wd)
CONV3D_MFMA = True
_MF_MAX_W = 8.0   # |w| * 2^12 < 2^15: the split weight's hi part stays in f16 range


def conv3d_mf_weights(w_t: torch.Tensor):
    """[Cin][27][Cout] 3x3x3 kernel (ops.conv3d layout) -> sa_conv3d_mf's B-fragment table, or
    None when the shape has no MFMA kernel or a weight is out of the split range."""
    _check(w_t, "w_t")
    cin, _, cout = w_t.shape
    n = int(N.lib().sa_conv3d_mf_weights_size(cin, cout))
    if n < 0 or not bool((w_t.abs() < _MF_MAX_W).all()):
        return None
    table = torch.empty((n,), device=w_t.device, dtype=torch.uint8)
    N.call("sa_conv3d_mf_weights", w_t.data_ptr(), cin, cout, table.data_ptr(), _stream(table))
    return table


def conv3d_mf(x: "VolAct", table: torch.Tensor, cout: int, slope: float = 0.01, stats: bool = True) -> "VolAct":
    """ops.conv3d at stride 1 for 8 -> 8 and 16 -> 16 on split-f16 MFMA (sa_conv3d_mf); the
    input must carry an InstanceNorm + LeakyReLU and no gate; table from conv3d_mf_weights."""
    _check(x.raw, "x")
    if x.norm is None or not x.act or x.gate is not None:
        raise ValueError("conv3d_mf: built for an InstanceNorm + LeakyReLU producer without gate")
    B, Cin, D, H, W = x.raw.shape
    out = torch.empty((B, cout, D, H, W), device=x.raw.device, dtype=torch.float32)
    parts = int(N.lib().sa_conv3d_mf_stat_parts(B, Cin, cout, D, H, W))
    if parts < 0:
        raise ValueError(f"conv3d_mf: no kernel for {Cin} -> {cout}")
    partial = torch.empty((B * cout * parts * 2,), device=out.device, dtype=torch.float64) if stats else None
    mean, rstd = x.norm
    N.call("sa_conv3d_mf", x.raw.data_ptr(), B, Cin, D, H, W, table.data_ptr(), cout, mean.data_ptr(),
           rstd.data_ptr(), slope, out.data_ptr(), _ptr(partial), _stream(out))
    norm = instnorm_finalize(partial, B * cout, parts, D * H * W) if stats else None
    return VolAct(out, norm, act=stats)


def conv3d_s1(x: "VolAct", w_wd: torch.Tensor, table, cout: int, slope: float = 0.01,
              stats: bool = True) -> "VolAct":
    """The hourglass's stride-1 conv: conv3d_mf where it applies (CONV3D_MFMA, a table, no gate),
    else conv3d_wd."""
    B, Cin, D, H, W = x.raw.shape
    if (CONV3D_MFMA and table is not None and x.gate is None and x.norm is not None and x.act
            and Cin * D * H * W * 4 < 2 ** 31 and D * H * W < 2 ** 30):
        return conv3d_mf(x, table, cout, slope, stats)
    return conv3d_wd(x, w_wd, cout, slope, stats)


def conv3d_s2mf_weights(w_t: torch.Tensor):
    """[16][27][32] 3x3x3 kernel (ops.conv3d layout) of the hourglass's stride-2 16 -> 32 conv ->
    sa_conv3d_s2mf's B-fragment table; None for other shapes or a weight out of the split range."""
    _check(w_t, "w_t")
    cin, _, cout = w_t.shape
    if (cin, cout) != (16, 32) or not bool((w_t.abs() < _MF_MAX_W).all()):
        return None
    table = torch.empty((int(N.lib().sa_conv3d_s2mf_weights_size()),), device=w_t.device, dtype=torch.uint8)
    N.call("sa_conv3d_s2mf_weights", w_t.data_ptr(), table.data_ptr(), _stream(table))
    return table


def conv3d_s2(x: "VolAct", w_t: torch.Tensor, table, cout: int, slope: float = 0.01, stats: bool = True) -> "VolAct":
    """The hourglass's stride-2 conv (down_layers[1][0]): 16 -> 32 on split-f16 MFMA
    (sa_conv3d_s2mf; CONV3D_MFMA, a table from conv3d_s2mf_weights, an InstanceNorm + LeakyReLU
    producer, optionally gated), else ops.conv3d at stride 2."""
    if (CONV3D_MFMA and table is not None and isinstance(x, VolAct) and x.norm is not None
            and x.act and x.raw.shape[1] == 16 and cout == 32):
        _check(x.raw, "x")
        B, Cin, D, H, W = x.raw.shape
        if Cin * D * H * W < 2 ** 31 and D * H * W < 2 ** 30:
            Do, Ho, Wo = (D - 1) // 2 + 1, (H - 1) // 2 + 1, (W - 1) // 2 + 1
            out = torch.empty((B, cout, Do, Ho, Wo), device=x.raw.device, dtype=torch.float32)
            parts = int(N.lib().sa_conv3d_s2mf_stat_parts(Do, Ho, Wo))
            partial = torch.empty((B * cout * parts * 2,), device=out.device, dtype=torch.float64) if stats else None
            mean, rstd = x.norm
            gl, gr = x.gate if x.gate is not None else (None, None)
            N.call("sa_conv3d_s2mf", x.raw.data_ptr(), B, D, H, W, table.data_ptr(), mean.data_ptr(),
                   rstd.data_ptr(), slope, _ptr(gl), _ptr(gr), out.data_ptr(), _ptr(partial), _stream(out))
            norm = instnorm_finalize(partial, B * cout, parts, Do * Ho * Wo) if stats else None
            return VolAct(out, norm, act=stats)
    return conv3d(x, w_t, cout, stride=2, slope=slope, stats=stats)


def _conv3d_onehot(x: OneHotVolume, w_t: torch.Tensor, cout: int, stride: int, stats: bool):
    _check(w_t, "w_t")
    B, nb, D, H, W = x.shape
    Do, Ho, Wo = (D - 1) // stride + 1, (H - 1) // stride + 1, (W - 1) // stride + 1
    out = torch.empty((B, cout, Do, Ho, Wo), device=x.device, dtype=torch.float32)
    parts = int(N.lib().sa_conv3d_onehot_stat_parts(Do, Ho, Wo))
    partial = torch.empty((B * cout * parts * 2,), device=out.device, dtype=torch.float64) if stats else None
    N.call("sa_conv3d_onehot", x.rec_l.data_ptr(), x.rec_r.data_ptr(), B, nb, D, H, W, stride, x.gain,
           w_t.data_ptr(), cout, out.data_ptr(), _ptr(partial), _stream(out))
    norm = instnorm_finalize(partial, B * cout, parts, Do * Ho * Wo) if stats else None
    return VolAct(out, norm, act=stats)


def conv3d_pointwise(x: "VolAct", w_t: torch.Tensor, cout: int, slope: float = 0.01) -> torch.Tensor:
    """1x1x1 conv of T(x.raw) (no statistics); w_t [Cin][Cout]."""
    _check(x.raw, "x")
    _check(w_t, "w_t")
    B, Cin, D, H, W = x.raw.shape
    out = torch.empty((B, cout, D, H, W), device=x.raw.device, dtype=torch.float32)
    a = x.args()
    N.call("sa_conv3d_pointwise", x.raw.data_ptr(), B, Cin, D, H, W, a[0], a[1], a[2], slope, a[3], a[4],
           w_t.data_ptr(), cout, out.data_ptr(), _stream(out))
    return out


def conv3d_pointwise_upcat(a: "VolAct", u: "VolAct", w_a: torch.Tensor, w_u: torch.Tensor, cout: int,
                           slope: float = 0.01) -> "VolAct":
    """1x1x1 conv over cat(T(a), trilinear_up(T(u))) -> VolAct(out, IN stats, act=True), as
    Wa.T(a) + up(Wu.T(u)) (two launches); w_a [Ca][Cout], w_u [Cu][Cout]."""
    if isinstance(a, OneHotVolume):
        p = conv3d_pointwise(u, w_u, cout, slope)
        B, _, D, H, W = a.shape
        _, _, Dp, Hp, Wp = p.shape
        out = torch.empty((B, cout, D, H, W), device=p.device, dtype=torch.float32)
        parts = int(N.lib().sa_conv3d_upcat_stat_parts(D, H, W))
        partial = torch.empty((B * cout * parts * 2,), device=out.device, dtype=torch.float64)
        N.call("sa_conv3d_pointwise_upcat_onehot", a.rec_l.data_ptr(), a.rec_r.data_ptr(), a.nbins, a.gain,
               p.data_ptr(), Dp, Hp, Wp, B, D, H, W, w_a.data_ptr(), cout, out.data_ptr(), partial.data_ptr(),
               _stream(out))
        return VolAct(out, instnorm_finalize(partial, B * cout, parts, D * H * W), act=True)
    _check(a.raw, "a")
    p = conv3d_pointwise(u, w_u, cout, slope)
    B, Ca, D, H, W = a.raw.shape
    _, _, Dp, Hp, Wp = p.shape
    out = torch.empty((B, cout, D, H, W), device=a.raw.device, dtype=torch.float32)
    parts = int(N.lib().sa_conv3d_upcat_stat_parts(D, H, W))
    partial = torch.empty((B * cout * parts * 2,), device=out.device, dtype=torch.float64)
    N.call("sa_conv3d_pointwise_upcat", a.raw.data_ptr(), Ca, *a.args(), p.data_ptr(), Dp, Hp, Wp, B, D,
           H, W, slope, w_a.data_ptr(), cout, out.data_ptr(), partial.data_ptr(), _stream(out))
    return VolAct(out, instnorm_finalize(partial, B * cout, parts, D * H * W), act=True)


def conv2d_small(x: torch.Tensor, w_t: torch.Tensor, bias: Optional[torch.Tensor], cout: int, ksize: int,
                 relu: bool = True) -> torch.Tensor:
    """Direct KxK conv (padding K//2) for few input channels; w_t pre-arranged [Cin][K][K][Cout]."""
    bs = _plane_bs(x, "x")
    B, Cin, H, W = x.shape
    out = torch.empty((B, cout, H, W), device=x.device, dtype=torch.float32)
    N.call("sa_conv2d_small", x.data_ptr(), bs, B, Cin, H, W, w_t.data_ptr(), _ptr(bias), cout, ksize,
           1 if relu else 0, out.data_ptr(), cout * H * W, _stream(x))
    _account("conv2d_small", 2.0 * B * cout * Cin * ksize * ksize * H * W)
    return out


# ----------------------------------------------------------------------- conv epilogues
ACT = {None: 0, "none": 0, "relu": 1, "tanh": 2}


def plane_stats(x: torch.Tensor, eps: float = 1e-5):
    """InstanceNorm2d statistics of every (b, c) plane -> (mean, rstd), each [B*C]."""
    bs = _plane_bs(x, "x")
    B, C, H, W = x.shape
    mean = torch.empty(B * C, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    N.call("sa_plane_stats", x.data_ptr(), bs, B, C, H * W, eps, mean.data_ptr(), rstd.data_ptr(), _stream(x))
    _account("norm_act", 4.0 * B * C * H * W)
    return mean, rstd


class Affine:
    """(x - m) * s + t with per-channel (``per_plane=False``) or per-(b, c) parameters;
    any of m / s / t may be None."""

    def __init__(self, m=None, s=None, t=None, per_plane: bool = False):
        self.m, self.s, self.t, self.per_plane = m, s, t, per_plane

    def args(self, C: int):
        return [_ptr(self.m), _ptr(self.s), _ptr(self.t), C if self.per_plane else 0]


def norm_act(x: torch.Tensor, aff: Optional[Affine] = None, act_in=None, skip: Optional[torch.Tensor] = None,
             skip_aff: Optional[Affine] = None, act_out=None, out: Optional[torch.Tensor] = None,
             skip_act=None) -> torch.Tensor:
    """out = act_out(act_in(aff(x)) + skip_act(skip_aff(skip))) in one pass (out may be x or a
    channel slice)."""
    xb = _plane_bs(x, "x")
    B, C, H, W = x.shape
    if out is None:
        out = torch.empty_like(x)
    if tuple(out.shape) != (B, C, H, W):
        raise RuntimeError(f"norm_act: out {tuple(out.shape)} != {(B, C, H, W)}")
    ob = _plane_bs(out, "out")
    sb = 0
    if skip is not None:
        if tuple(skip.shape) != (B, C, H, W):
            raise RuntimeError("norm_act: skip shape mismatch")
        sb = _plane_bs(skip, "skip")
    a = (aff or Affine()).args(C)
    sa_ = (skip_aff or Affine()).args(C)
    N.call("sa_norm_act", x.data_ptr(), xb, B, C, H * W, *a, ACT[act_in], _ptr(skip), sb, *sa_, ACT[skip_act],
           ACT[act_out],
           out.data_ptr(), ob, _stream(x))
    _account("norm_act", 4.0 * B * C * H * W * (3 if skip is not None else 2))
    return out


def conv2d_k3_narrow(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """3x3 / pad 1 conv to 2 channels (weight [2, Cin, 3, 3] as stored by nn.Conv2d)."""
    bs = _plane_bs(x, "x")
    _check(weight, "weight")
    B, Cin, H, W = x.shape
    cout = weight.shape[0]
    out = torch.empty((B, cout, H, W), device=x.device, dtype=torch.float32)
    N.call("sa_conv2d_k3_narrow", x.data_ptr(), bs, B, Cin, H, W, weight.data_ptr(), _ptr(bias), cout,
           out.data_ptr(), cout * H * W, _stream(x))
    _account("conv2d_narrow", 4.0 * B * (Cin + cout) * H * W)   # the input read once, the output written
    return out


class WinoFilters:
    """Derived filters of one 3x3 conv for the fused Winograd kernels: ``u2`` for F(2x2,3x3)
    (conv2d_wino.hip), ``u4`` for F(4x4,3x3) (conv2d_wino4.hip) in 32-channel blocks and ``u4s`` as
    the split F(4x4) kernel's f16 hi/lo pairs (None unless W4_SPLIT when derived)."""
    __slots__ = ("u2", "u4", "u4s", "cin", "cout")

    def __init__(self, u2: torch.Tensor, u4: torch.Tensor, cin: int, cout: int, u4s: Optional[torch.Tensor] = None):
        self.u2, self.u4, self.u4s, self.cin, self.cout = u2, u4, u4s, cin, cout


# False keeps every 3x3 conv on the F(2x2,3x3) kernel (set by A/B scripts and tests)
_WINO4 = True
# F(4x4) launches of the default shape on the split kernel (block_shape 6): the Winograd-domain
# products on v_mfma_f32_16x16x16_f16 with f16 hi/lo operand pairs (22 significant bits, exact
# f16 x f16 products, fp32 accumulation) instead of fp32 MFMA: 1.06-1.22x per conv, 54.3 -> 60.4
# pairs/s at configs[1] with EPE vs the reference 1.78e-5 (fp32 MFMA: 1.84e-5)
W4_SPLIT = True
# (round 5 built a split-f16 implicit-GEMM 3x3 conv on 16x16x32 MFMA, conv2d_igemm.hip: 0.88-1.02x
# F(4x4) per conv at the model's shapes and slower in the forward, so it was off by default; round 6
# deleted it)
# the split filters need |U * 2^12| < 65504; |U| <= max |weight| for F(4x4,3x3)'s G
_W4_SPLIT_WMAX = 15.99
# the direct convs (stems, stride-2 + 1x1) with split products (sa_conv_direct_split), derived
# by conv_direct_weights as int32-held (hi, lo) pairs: 1.4-1.9x per conv, conv2d_direct 4.36 ->
# 2.8 ms/step, 60.0 -> 61.9 pairs/s, EPE vs the reference 1.74e-5
DIRECT_SPLIT = True


def split_range_ok(*weights: Optional[torch.Tensor]) -> bool:
    """Whether the split kernels' f16 filter pairs hold these weights: |w * 2^12| < 65504 (and the
    F(4x4,3x3) transform keeps |U| <= max |w|), i.e. |w| < 16.  Otherwise the conv keeps its fp32
    filters and runs on the fp32-product kernels (e.g. an eval-BatchNorm-folded conv of a trained
    checkpoint with a large gamma / sqrt(var))."""
    return all(w is None or float(w.abs().max()) < _W4_SPLIT_WMAX for w in weights)


def wino_weights(weight: torch.Tensor) -> WinoFilters:
    """[Cout, Cin, 3, 3] -> Winograd filters (fp64 transforms, rounded once): U2 [16][Cin/8][4][Cout][2]
    and U4 [Cout/32][Cin/8][36][2][4][32], each in a flat container."""
    _check(weight, "weight")
    Cout, Cin = weight.shape[:2]
    u2 = torch.empty((16 * Cin * Cout,), device=weight.device, dtype=torch.float32)
    N.call("sa_conv2d_wino_weights", weight.data_ptr(), Cout, Cin, u2.data_ptr(), _stream(weight))
    u4 = torch.empty((36 * Cin * Cout,), device=weight.device, dtype=torch.float32)
    N.call("sa_conv2d_wino4_weights", weight.data_ptr(), Cout, Cin, u4.data_ptr(), _stream(weight))
    u4s = None
    # (a conv whose filters exceed the split kernel's f16 range keeps u4s = None: its launches run
    # the fp32-product kernel, conv2d_k3_multi)
    if W4_SPLIT and Cout % 32 == 0 and Cin % 8 == 0 and split_range_ok(weight):
        u4s = torch.empty((36 * Cin * Cout,), device=weight.device, dtype=torch.int32)
        N.call("sa_conv2d_wino4_weights_split", weight.data_ptr(), Cout, Cin, u4s.data_ptr(), _stream(weight))
    return WinoFilters(u2, u4, Cin, Cout, u4s)


# largest Cin of an F(4x4,3x3) launch with an input transform (its (scale, shift) table fills the
# 8-wave block's spare LDS)
_WINO4_AFF_CIN = 256


def _wino4_ok(x: torch.Tensor, in_aff=None, in_act=None, out: Optional[torch.Tensor] = None,
              width: Optional[int] = None, **_) -> bool:
    """F(4x4,3x3) kernel preconditions: W % 4 == 0 (the pitch of pitched planes), 16-byte aligned
    planes; an input transform (the producer's norm, ReLU or none) for Cin <= _WINO4_AFF_CIN and
    not on pitched planes (it would turn their zero pad columns into t)."""
    if (in_aff is not None or in_act is not None) and (x.shape[1] > _WINO4_AFF_CIN or ACT[in_act] > 1
                                                      or (width is not None and width != x.shape[3])):
        return False
    return (x.shape[3] % 4 == 0 and x.data_ptr() % 16 == 0
            and x.stride(0) % 4 == 0 and (out is None or (out.data_ptr() % 16 == 0 and out.stride(0) % 4 == 0)))


def _wino4_blocks(x: torch.Tensor, U: "WinoFilters", **_) -> int:
    """Workgroups of the F(4x4,3x3) launch for one conv (conv2d_wino4.hip's geometry chooser:
    16 x 64 or 8 x 128 output pixels per block, whichever pads less; 32 channels per block)."""
    B, _, H, W = x.shape
    a16 = -(-W // 64) * 64 * -(-H // 16) * 16
    a32 = -(-W // 128) * 128 * -(-H // 8) * 8
    bh, bw = (8, 128) if a32 < a16 else (16, 64)
    return B * -(-H // bh) * -(-W // bw) * (U.cout // 32)


# below this many workgroups per launch the F(2x2) kernel's four times as many, smaller blocks
# fill the chip better than F(4x4)'s (measured on the update block's convs: 384 with the fp32
# F(4x4) kernel; with the split kernel 128 is 0.4 ms/step faster in the forward than 384 or
# 256, bench.py --wino4-min-blocks, two interleaved passes)
_WINO4_MIN_BLOCKS = 128


def _wino_problem(x: torch.Tensor, U: WinoFilters, bias: Optional[torch.Tensor] = None, relu: bool = False,
                  out: Optional[torch.Tensor] = None, in_aff: Optional[Affine] = None, in_act=None,
                  stats: bool = False, f4: bool = False, out_cout: Optional[int] = None,
                  width: Optional[int] = None, split: bool = False,
                  skip: Optional[torch.Tensor] = None, skip_s: Optional[torch.Tensor] = None,
                  skip_t: Optional[torch.Tensor] = None, skip_act=None, out_act=None):
    """out_cout: channels of ``out`` when the epilogue writes fewer than Cout there (gate mode 1).
    width: the image width when x (and out, and the gate planes) are PITCHED planes [.., H, P]
    whose columns width .. P - 1 are zero (F(4x4) only; the outputs' pad columns stay zero).
    skip: the residual epilogue (F(4x4) only): out = out_act(act(conv + bias) + skip_act(skip *
    skip_s + skip_t)), skip_s / skip_t per output channel (SaWinoProblem skip)."""
    bs = _plane_bs(x, "x")
    if not isinstance(U, WinoFilters):
        raise RuntimeError("conv2d_k3: U must come from ops.wino_weights")
    B, Cin, H, P = x.shape
    W = P if width is None else width
    if not 0 < W <= P:
        raise RuntimeError(f"conv2d_k3: width {W} outside the plane pitch {P}")
    if W != P and not f4:
        raise RuntimeError("conv2d_k3: pitched planes need the F(4x4,3x3) kernel")
    Cout = U.cout
    if U.cin != Cin:
        raise RuntimeError(f"conv2d_k3: U has {U.cin} input channels, x has {Cin}")
    if out is None:
        alloc = torch.zeros if W != P else torch.empty
        out = alloc((B, out_cout or Cout, H, P), device=x.device, dtype=torch.float32)
    if tuple(out.shape) != (B, out_cout or Cout, H, P):
        raise RuntimeError("conv2d_k3: out shape mismatch")
    m, s, t, ps = (in_aff or Affine()).args(Cin)
    parts_fn = N.lib().sa_conv2d_k3_wino4_stat_parts if f4 else N.lib().sa_conv2d_k3_wino_stat_parts
    parts = int(parts_fn(H, W)) if stats else 0
    partial = torch.empty((B * Cout * parts * 2,), device=x.device, dtype=torch.float64) if stats else None
    Uf = (U.u4s if split else U.u4) if f4 else U.u2
    prob = N.SaWinoProblem(x.data_ptr(), bs, B, Cin, H, W, Uf.data_ptr(), Cout, _ptr(bias),
                           1 if relu else 0, m, s, t, ps, ACT[in_act], out.data_ptr(), _plane_bs(out, "out"),
                           _ptr(partial), P if P != W else 0)
    if skip is not None:
        if not f4 or stats:
            raise RuntimeError("conv2d_k3: the residual epilogue needs the F(4x4) kernel and no statistics")
        if tuple(skip.shape) != (B, Cout, H, P) or skip.stride(1) != H * P:
            raise RuntimeError(f"conv2d_k3: skip must be [{B}, {Cout}, {H}, {P}] planes")
        for v in (skip_s, skip_t):
            if v is not None:
                _check(v, "skip_s / skip_t")
        prob.skip, prob.skip_bs = skip.data_ptr(), _plane_bs(skip, "skip")
        prob.skip_s, prob.skip_t = _ptr(skip_s), _ptr(skip_t)
        prob.skip_act, prob.out_act = ACT[skip_act], ACT[out_act]
    # Winograd-domain products actually executed: 36 per 4x4 tile (F4) or 16 per 2x2 tile (F2)
    # per (Cin, Cout) pair
    if f4:
        _account("conv2d_wino4", 2.0 * 36 * Cin * Cout * B * ((H + 3) // 4) * ((W + 3) // 4))   # logical W
    else:
        _account("conv2d_wino", 2.0 * 16 * Cin * Cout * B * ((H + 1) // 2) * ((W + 1) // 2))
    fin = (lambda: (out, instnorm_finalize(partial, B * Cout, parts, H * W))) if stats else (lambda: out)
    return prob, fin


def wino4_applies(x: torch.Tensor, U: "WinoFilters", *more) -> bool:
    """Whether conv2d_k3 of x (and of the further (x, U) pairs in ``more``, in one
    conv2d_k3_multi launch) without an input transform runs on the F(4x4,3x3) kernel."""
    pairs = [(x, U)] + list(more)
    return (_WINO4 and all(_wino4_ok(a) for a, _ in pairs)
            and sum(_wino4_blocks(a, u) for a, u in pairs) >= _WINO4_MIN_BLOCKS)


def _gate_epilogue(p: dict) -> "N.SaGateEpilogue":
    """ConvGRU gate epilogue of one problem (sa_conv2d_k3_wino4_multi_gate):
    gate=dict(mode=1, ctx=, h=, out2=): out = z, out2 = r*h for a conv over cat(h, x) with
    Cout = 2*Ch (convz | convr); gate=dict(mode=2, ctx=, h=, z=, add=): out = the new state
    (1 - z) h + z tanh(add + conv + ctx) for convq's r*h part (out may be h itself)."""
    g = p["gate"]
    mode = g["mode"]
    B, _, H, W = p["x"].shape   # (the plane pitch for pitched problems: every gate plane shares it)
    Cout = p["U"].cout
    Ch = Cout // 2 if mode == 1 else Cout
    ctx, h = g["ctx"], g["h"]
    if ctx.shape[0] != B or ctx.shape[1] < Cout or tuple(ctx.shape[2:]) != (H, W):
        raise RuntimeError("gate: ctx must be [B, >= Cout, H, W]")
    if tuple(h.shape) != (B, Ch, H, W):
        raise RuntimeError(f"gate: h must be {(B, Ch, H, W)}")
    e = N.SaGateEpilogue(mode, ctx.data_ptr(), _plane_bs(ctx, "ctx"), h.data_ptr(), _plane_bs(h, "h"))
    if mode == 1:
        o2 = g["out2"]
        if tuple(o2.shape) != (B, Ch, H, W):
            raise RuntimeError("gate: out2 shape mismatch")
        e.out2, e.out2_bs = o2.data_ptr(), _plane_bs(o2, "out2")
    elif mode == 2:
        for k in ("z", "add"):
            t = g[k]
            if tuple(t.shape) != (B, Ch, H, W):
                raise RuntimeError(f"gate: {k} shape mismatch")
            setattr(e, k, t.data_ptr())
            setattr(e, k + "_bs", _plane_bs(t, k))
    else:
        raise RuntimeError(f"gate: mode {mode}")
    return e


# (round 6: fnet.layer1's plain 64 -> 64 shape measured 1.03 ms on the fp32-product kernel against
# 1.13 ms split, but with its layer-1 launches on fp32 products the forward was slower, 61.0 / 61.3 vs
# 60.7 ms/step in two interleaved passes: the split kernel stays on every F(4x4) launch)

# the split kernels' f16 range guards (False: no overflow check or recompute: A/B timing only)
SPLIT_GUARD = True


def _wino4_launch(n: int, arr, gates, shape: int, x: torch.Tensor) -> None:
    """sa_conv2d_k3_wino4_launch; the split shape (6) with its range guard (an overflowed block
    recomputes itself on fp32 products inside the launch)."""
    N.call("sa_conv2d_k3_wino4_launch", n, ctypes.addressof(arr), ctypes.addressof(gates), shape,
           1 if (shape == 6 and SPLIT_GUARD) else 0, _stream(x))


def conv2d_k3_multi(*problems, small_blocks: bool = False) -> list:
    """Independent conv2d_k3 calls (each a dict of conv2d_k3's keyword arguments) in ONE launch:
    their blocks share the grid, so each conv's partly filled last round of blocks is filled by
    the others.  On the F(4x4,3x3) kernel when every problem meets its preconditions; a group
    that mixes eligible and ineligible problems is split into an F(4x4) and an F(2x2) launch;
    on F(2x2,3x3) all must agree on Cout % 64 == 0 and on having an input transform or not.
    A problem with a ``gate`` (_gate_epilogue) puts the launch on F(4x4,3x3) whatever its size.
    small_blocks: F(4x4)'s small block shape (two blocks per CU) for this launch."""
    if not 1 <= len(problems) <= 8:
        raise RuntimeError("conv2d_k3_multi: 1..8 convolutions per launch")
    gated = any(p.get("gate") for p in problems)
    plain = [{k: v for k, v in p.items() if k != "gate"} for p in problems]
    for p, q in zip(problems, plain):
        if p.get("gate") and p["gate"]["mode"] == 1:
            q["out_cout"] = p["U"].cout // 2   # z only: r*h goes to the gate's out2
    oks = [_WINO4 and _wino4_ok(**p) for p in plain]
    if any(oks) and not all(oks):
        # a mixed group: the problems F(4x4) cannot take (W % 4 != 0, unaligned planes) go to a
        # launch of their own instead of demoting the whole group to F(2x2) — unless the F(4x4)
        # part is too small for F(4x4) anyway (then one F(2x2) launch of all of them)
        four = [i for i, k in enumerate(oks) if k]
        if gated or sum(_wino4_blocks(**plain[i]) for i in four) >= _WINO4_MIN_BLOCKS:
            two = [i for i, k in enumerate(oks) if not k]
            res = [None] * len(problems)
            for idx in (four, two):
                for i, r in zip(idx, conv2d_k3_multi(*[problems[i] for i in idx], small_blocks=small_blocks)):
                    res[i] = r
            return res
    ok4 = all(oks)
    if gated and not ok4:
        raise RuntimeError("conv2d_k3_multi: gate epilogues need the F(4x4,3x3) kernel (gate_f4_ok)")
    has_skip = any(p.get("skip") is not None for p in plain)
    if has_skip and not ok4:
        raise RuntimeError("conv2d_k3_multi: a residual epilogue needs the F(4x4,3x3) kernel")
    f4 = ok4 and (gated or has_skip or sum(_wino4_blocks(**p) for p in plain) >= _WINO4_MIN_BLOCKS)
    aff = any(p.get("in_aff") is not None or p.get("in_act") is not None for p in plain)
    if gated and aff:
        raise RuntimeError("conv2d_k3_multi: an input transform and a gate epilogue in one launch")
    split = f4 and W4_SPLIT and not small_blocks and all(p["U"].u4s is not None for p in plain)
    built = [_wino_problem(**p, f4=f4, split=split) for p in plain]
    arr = (N.SaWinoProblem * len(built))(*[b[0] for b in built])
    if f4 and (gated or small_blocks or split):
        gates = (N.SaGateEpilogue * len(built))(*[_gate_epilogue(p) if p.get("gate") else N.SaGateEpilogue()
                                                  for p in problems])
        _wino4_launch(len(built), arr, gates, 2 if small_blocks else 6 if split else 0, problems[0]["x"])
    else:
        N.call("sa_conv2d_k3_wino4_multi" if f4 else "sa_conv2d_k3_wino_multi", len(built), ctypes.addressof(arr),
               _stream(problems[0]["x"]))
    return [b[1]() for b in built]


def flow_head_update(h: torch.Tensor, U1: "WinoFilters", b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
                     coords_x: torch.Tensor, flow: Optional[torch.Tensor] = None) -> bool:
    """The flow head (update.py:98-110: conv2(relu(conv1(h)))) fused with the coordinate update
    (stereoanywhere.py:283-285: coords_x += delta_flow[:, 0]; the model reads conv2's channel 0
    only): conv1 on the F(4x4,3x3) kernel with its epilogue summing conv2's channel-0 taps over each
    block's channels (gate mode 3), then sa_flow_head_reduce; conv1's [B, Cout, H, W] output is
    never written.  flow: the [B, 2, H, W] flow planes to refresh (as flow_update).  Returns False
    (nothing launched) where the F(4x4) kernel does not take h: the caller then runs
    conv2d_k3 + conv2d_k3_narrow + flow_update."""
    B, Cin, H, W = h.shape
    if not (_WINO4 and _wino4_ok(h) and U1.cout % 32 == 0 and U1.cin == Cin):
        return False
    split = W4_SPLIT and U1.u4s is not None
    per = int(N.lib().sa_flow_head_part_size(1, U1.cout, H, W))
    part = torch.empty((B * per,), device=h.device, dtype=torch.float32)
    w2c = w2[0].contiguous()    # conv2's channel-0 filter [Cout][3][3]
    _check(w2c, "w2")
    _check(b2, "b2")
    Uf = U1.u4s if split else U1.u4
    prob = N.SaWinoProblem(h.data_ptr(), _plane_bs(h, "h"), B, Cin, H, W, Uf.data_ptr(), U1.cout, _ptr(b1), 1,
                           None, None, None, 0, 0, part.data_ptr(), 0, None, 0)
    gate = N.SaGateEpilogue(3)
    gate.head_w, gate.head_part, gate.head_part_bs = w2c.data_ptr(), part.data_ptr(), per
    _account("conv2d_wino4", 2.0 * 36 * Cin * U1.cout * B * ((H + 3) // 4) * ((W + 3) // 4))
    _wino4_launch(1, prob, gate, 6 if split else 0, h)
    _check(coords_x, "coords_x")
    N.call("sa_flow_head_reduce", part.data_ptr(), B, U1.cout, H, W, b2.data_ptr(), coords_x.data_ptr(),
           _ptr(flow), 0 if flow is None else _plane_bs(flow, "flow"), None, 0, _stream(h))
    _account("gru_plumbing", 4.0 * B * (per + H * W * (2 + (2 if flow is not None else 0))))
    return True


def gate_f4_ok(*xs: torch.Tensor) -> bool:
    """Whether GRU gate epilogues can run on convs of these inputs (F(4x4,3x3) preconditions)."""
    return _WINO4 and all(_wino4_ok(x) for x in xs)


def conv2d_k3(x: torch.Tensor, U: torch.Tensor, bias: Optional[torch.Tensor] = None, relu: bool = False,
              out: Optional[torch.Tensor] = None, in_aff: Optional[Affine] = None, in_act=None,
              stats: bool = False, **residual):
    """3x3 / pad 1 conv via fused Winograd (U from wino_weights); + bias, optional ReLU.
    in_aff / in_act: the producer's norm + activation applied to x while it is loaded.
    stats: also return the output's InstanceNorm (mean, rstd) per (image, channel).
    residual: skip / skip_s / skip_t / skip_act / out_act of _wino_problem's residual epilogue."""
    return conv2d_k3_multi(dict(x=x, U=U, bias=bias, relu=relu, out=out, in_aff=in_aff, in_act=in_act,
                                stats=stats, **residual))[0]


# the 1x1 convs (fnet's output conv, the mask head's 1x1) on sa_conv1x1 (False: F.conv2d, A/B runs)
CONV1X1 = True


def conv1x1_weights(weight: torch.Tensor) -> Optional[torch.Tensor]:
    """[Cout, Cin, 1, 1] (or [Cout, Cin]) -> the split weights of sa_conv1x1 (f16 hi / lo planes of
    w * 2^12), or None where the kernel does not take the conv (|w| >= 16, Cin % 32 != 0): the
    caller keeps F.conv2d."""
    w = weight.detach().reshape(weight.shape[0], -1).contiguous()
    _check(w, "weight")
    Cout, Cin = w.shape
    if not CONV1X1 or Cin % 32 or not split_range_ok(w):
        return None
    out = torch.empty((int(N.lib().sa_conv1x1_weights_size(Cout, Cin)),), device=w.device, dtype=torch.uint8)
    N.call("sa_conv1x1_weights", w.data_ptr(), Cout, Cin, out.data_ptr(), _stream(w))
    return out


def conv1x1(x: torch.Tensor, wsplit: torch.Tensor, Cout: int, bias: Optional[torch.Tensor] = None,
            scale: float = 1.0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """scale * (F.conv2d(x, w, bias)) for a 1x1 stride-1 conv on split-f16 MFMA (sa_conv1x1; weights
    from conv1x1_weights): the feature encoder's output conv and the mask head's 1x1."""
    bs = _plane_bs(x, "x")
    B, Cin, H, W = x.shape
    if out is None:
        out = torch.empty((B, Cout, H, W), device=x.device, dtype=torch.float32)
    if tuple(out.shape) != (B, Cout, H, W):
        raise RuntimeError("conv1x1: out shape mismatch")
    if bias is not None:
        _check(bias, "bias")
    N.call("sa_conv1x1", x.data_ptr(), bs, B, Cin, H, W, wsplit.data_ptr(), Cout, _ptr(bias), float(scale),
           out.data_ptr(), _plane_bs(out, "out"), _stream(x))
    _account("conv1x1", 4.0 * B * (Cin + Cout) * H * W)   # bytes: x read once, out written once
    return out


# ----------------------------------------------------------------------- tiled harness (tiler.hip)
def tile_gather_pad(src: torch.Tensor, origins: List[Tuple[int, int]], th: int, tw: int, pad) -> torch.Tensor:
    """torch.cat of the [1, C, th, tw] views of src [1, C, H, W] at origins (row, column), then
    F.pad(pad = [left, right, top, bottom], mode="replicate"), in one launch (sa_tile_gather_pad)."""
    _check(src, "src")
    _, C, H, W = src.shape
    pl, pr, pt, pb = pad
    org = torch.tensor([v for o in origins for v in o], dtype=torch.int32).to(src.device, non_blocking=True)
    out = torch.empty((len(origins), C, th + pt + pb, tw + pl + pr), device=src.device, dtype=torch.float32)
    N.call("sa_tile_gather_pad", src.data_ptr(), C, H, W, org.data_ptr(), len(origins), th, tw, pt, pb, pl, pr,
           out.data_ptr(), _stream(src))
    org.record_stream(torch.cuda.current_stream(src.device))
    return out


def tile_stitch(disp: torch.Tensor, tiles: List[Tuple[int, int, int]], wgt: torch.Tensor, H: int, W: int,
                finalize: bool, num: torch.Tensor, den: torch.Tensor) -> None:
    """The stitching loop of TileWrapper.forward in one launch (sa_tile_stitch): disp [n, 1, th, tw]
    (a view with any row pitch), tiles = (row, column, slot in disp) in the reference's order."""
    n, _, th, tw = disp.shape
    if disp.stride(3) != 1:
        raise RuntimeError("tile_stitch: disp rows must be contiguous")
    _check(wgt, "wgt")
    _check(num, "num")
    _check(den, "den")
    tl = torch.tensor([v for t in tiles for v in t], dtype=torch.int32).to(disp.device, non_blocking=True)
    N.call("sa_tile_stitch", disp.data_ptr(), disp.stride(0), disp.stride(2), tl.data_ptr(), len(tiles), th, tw,
           wgt.data_ptr(), H, W, 1 if finalize else 0, num.data_ptr(), den.data_ptr(), _stream(disp))
    tl.record_stream(torch.cuda.current_stream(disp.device))


def conv_direct_weights(weight: torch.Tensor, stride: int, with_ds: bool = False,
                        split: Optional[bool] = None) -> torch.Tensor:
    """[Cout, Cin, K, K] -> the direct-conv kernel's chunked layout (sa_conv_direct_weights).
    with_ds: the weight is the 1x1 downsample fused into a stride-``stride`` 3x3 launch.
    split: the split kernel's (hi, lo) pairs (default: DIRECT_SPLIT where split_range_ok; a 3x3
    and its fused downsample must agree, encoders.direct_table decides for both)."""
    _check(weight, "weight")
    Cout, Cin, K, _ = weight.shape
    n = int(N.lib().sa_conv_direct_weights_size(Cout, Cin, K, stride, 1 if with_ds else 0))
    if n < 0:
        raise RuntimeError(f"conv_direct_weights: no kernel for K={K} stride={stride} Cout={Cout}")
    out = torch.empty((n,), device=weight.device, dtype=torch.float32)
    N.call("sa_conv_direct_weights", weight.data_ptr(), Cout, Cin, K, stride, 1 if with_ds else 0, out.data_ptr(),
           _stream(weight))
    if split is None:
        split = DIRECT_SPLIT and split_range_ok(weight)
    elif split and not split_range_ok(weight):
        raise RuntimeError("conv_direct_weights: |weight| >= 16 exceeds the split kernel's f16 range")
    if split:   # the split kernel's (hi, lo) pairs: an int32 container marks them
        sp = torch.empty((n,), device=weight.device, dtype=torch.int32)
        N.call("sa_conv_direct_weights_split", out.data_ptr(), n, sp.data_ptr(), _stream(weight))
        return sp
    return out


def conv_direct_close_supported(K: int, stride: int, Cout: int) -> bool:
    """Whether conv_direct takes ``close`` for this conv (sa_conv_direct_close_supported)."""
    return bool(N.lib().sa_conv_direct_close_supported(K, stride, Cout))


def conv_direct(x: torch.Tensor, wg: torch.Tensor, K: int, stride: int, Cout: int,
                wd: Optional[torch.Tensor] = None, stats: bool = False, close=None):
    """KxK conv (padding K//2, no bias) on fp32 MFMA: the 7x7 stems and the stride-2 3x3 conv
    with its fused 1x1 stride-2 downsample (wd).  Returns [out, (out_ds)] and, with stats,
    the InstanceNorm (mean, rstd) of each output after it.
    close = (skip, mean, rstd): x is a residual block's raw conv2 output and the conv's input is
    the block's output relu(relu((x - mean) * rstd) + skip), formed while staging
    (sa_conv_direct_close; conv_direct_close_supported)."""
    bs = _plane_bs(x, "x")
    if wg.dtype == torch.int32:   # split (hi, lo) pairs (conv_direct_weights under DIRECT_SPLIT)
        if wg.device.type != "cuda" or not wg.is_contiguous():
            raise RuntimeError("conv_direct: wg must be a contiguous GPU tensor")
    else:
        _check(wg, "wg")
    B, Cin, H, W = x.shape
    p = K // 2
    Ho, Wo = (H + 2 * p - K) // stride + 1, (W + 2 * p - K) // stride + 1
    out = torch.empty((B, Cout, Ho, Wo), device=x.device, dtype=torch.float32)
    out_ds = torch.empty_like(out) if wd is not None else None
    parts = int(N.lib().sa_conv_direct_stat_parts(Ho, Wo)) if stats else 0

    def part():
        return torch.empty((B * Cout * parts * 2,), device=x.device, dtype=torch.float64) if stats else None
    pa, pd = part(), (part() if wd is not None else None)
    split = wg.dtype == torch.int32
    if wd is not None and (wd.dtype == torch.int32) != split:
        raise RuntimeError("conv_direct: wg and wd must both be split or both fp32 (conv_direct_weights)")
    if close is not None:
        skip, mean, rstd = close
        if tuple(skip.shape) != (B, Cin, H, W):
            raise RuntimeError("conv_direct: close skip shape mismatch")
        for t, nm in ((mean, "mean"), (rstd, "rstd")):
            _check(t, nm)
            if t.numel() != B * Cin:
                raise RuntimeError(f"conv_direct: close {nm} must have B*Cin entries")
        N.call("sa_conv_direct_close", x.data_ptr(), bs, skip.data_ptr(), _plane_bs(skip, "skip"), mean.data_ptr(),
               rstd.data_ptr(), B, Cin, H, W, K, stride, wg.data_ptr(), _ptr(wd), int(split), Cout, out.data_ptr(),
               Cout * Ho * Wo, _ptr(out_ds), Cout * Ho * Wo, _ptr(pa), _ptr(pd), _stream(x))
    else:
        N.call("sa_conv_direct_split" if split else "sa_conv_direct", x.data_ptr(), bs, B, Cin, H, W, K, stride,
               wg.data_ptr(), _ptr(wd), Cout, out.data_ptr(), Cout * Ho * Wo, _ptr(out_ds), Cout * Ho * Wo, _ptr(pa),
               _ptr(pd), _stream(x))
    # products executed: the stem's channels padded to the kernel's chunk of 4
    cin_x = -(-Cin // 4) * 4 if K == 7 else Cin
    _account("conv2d_direct", 2.0 * B * Cout * cin_x * K * K * Ho * Wo
             + (2.0 * B * Cout * Cin * Ho * Wo if wd is not None else 0))
    res = [out] + ([out_ds] if wd is not None else [])
    if stats:
        res.append([instnorm_finalize(q, B * Cout, parts, Ho * Wo) for q in (pa, pd) if q is not None])
    return res


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("annotations", "ctypes", "math", "torch")]
