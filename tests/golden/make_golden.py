"""Generate the golden vectors under tests/golden/ by running the REFERENCE here.

Test infrastructure only; run in the build container (where /root/reference is
mounted), never on the GPU box:

    python tests/golden/make_golden.py

The reference is pure PyTorch. It imports here once five third-party modules
that are absent from this image are stubbed:

* ``cv2``, ``timm``, ``torchvision``(+``.ops``) — import-only on the path
  (stereoanywhere.py:8, submodule.py:6, dcn.py:2);
* ``opt_einsum`` — imported, never called (update.py:4);
* ``kornia.filters.spatial_gradient`` — the one that executes (utils.py:3,74).
  kornia is unpinned (requirements.txt:3) and absent, so it is restated below
  as kornia's ``mode='diff', order=1, normalized=False`` path: replicate pad by
  one, cross-correlate with [-1, 0, 1] along x and y.  Parity across this
  boundary is therefore pinned to this restatement, not to kornia itself.

Weights are the seeded ones of ``stereoanywhere_amd.synth`` (no checkpoint is
available offline); inputs are ``synth.synthetic_pair`` and their sha256 is
stored next to the outputs so the consumer can check it regenerated the same
bytes.
"""
from __future__ import annotations

import json
import os
import sys
import types
import warnings

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from stereoanywhere_amd import synth  # noqa: E402

# Flag set of the published runs (README.md:314-321; run_test.py:62-74).
REF_ARGS = dict(
    n_downsample=2, n_additional_hourglass=0, volume_channels=8, vol_downsample=0,
    vol_n_masks=8, use_truncate_vol=True, mirror_conf_th=0.98, mirror_attenuation=0.9,
    use_aggregate_stereo_vol=False, use_aggregate_mono_vol=True, normal_gain=10, lrc_th=1.0,
    corr_implementation="reg",
)


def _install_stubs() -> None:
    for name in ("cv2", "timm", "torchvision", "torchvision.ops"):
        sys.modules.setdefault(name, types.ModuleType(name))
    oe = types.ModuleType("opt_einsum")
    oe.contract = torch.einsum
    sys.modules["opt_einsum"] = oe

    def spatial_gradient(inp, mode="diff", order=1, normalized=False):
        assert mode == "diff" and order == 1 and not normalized
        b, c, h, w = inp.shape
        kx = torch.tensor([[0.0, 0.0, 0.0], [-1.0, 0.0, 1.0], [0.0, 0.0, 0.0]], dtype=inp.dtype)
        k = torch.stack([kx, kx.t()])[:, None]
        x = F.pad(inp.reshape(b * c, 1, h, w), [1, 1, 1, 1], mode="replicate")
        return F.conv2d(x, k).reshape(b, c, 2, h, w)

    kornia = types.ModuleType("kornia")
    filters = types.ModuleType("kornia.filters")
    filters.spatial_gradient = spatial_gradient
    kornia.filters = filters
    sys.modules["kornia"] = kornia
    sys.modules["kornia.filters"] = filters


def _load_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    import models.stereoanywhere.stereoanywhere as sa_mod  # noqa
    import models.stereoanywhere.utils.utils as ut  # noqa
    import models.stereoanywhere.corr as corr_mod  # noqa
    return sa_mod, ut, corr_mod


def _np(t):
    return t.detach().cpu().float().numpy().copy() if torch.is_tensor(t) else np.asarray(t)


def build_model(sa_mod):
    torch.manual_seed(0)
    model = sa_mod.StereoAnywhere(dict(REF_ARGS)).eval()
    synth.load_seeded_weights(model, seed=0)
    return model


def run_capture(sa_mod, ut, corr_mod, model, pair, iters, capture_all):
    """Run the reference forward with wrappers that record every hot-path intermediate."""
    rec = {}
    calls = {}

    def tap(name, fn):
        def w(*a, **k):
            out = fn(*a, **k)
            n = calls.get(name, 0)
            calls[name] = n + 1
            if capture_all:
                key = f"{name}.{n}"
                for i, x in enumerate(a):
                    if torch.is_tensor(x):
                        rec[f"{key}.in{i}"] = _np(x)
                for kk, x in k.items():
                    if torch.is_tensor(x):
                        rec[f"{key}.kw_{kk}"] = _np(x)
                outs = out if isinstance(out, (tuple, list)) else (out,)
                for i, x in enumerate(outs):
                    if torch.is_tensor(x):
                        rec[f"{key}.out{i}"] = _np(x)
            return out
        return w

    saved = {}
    names = ["estimate_normals", "generate_masks", "estimate_left_disparity", "estimate_right_disparity",
             "estimate_left_confidence", "estimate_right_confidence", "softlrc", "weighted_lsq",
             "handcrafted_mirror_detector", "truncate_corr_volume_v2", "convex_upflow", "initialize_flow"]
    for n in names:
        saved[n] = getattr(sa_mod, n)
        setattr(sa_mod, n, tap(n, saved[n]))

    # torch.linalg.lstsq (utils.py:381) is not deterministic on the multi-threaded CPU
    # LAPACK: at cfg1 its fp32 shift moved by 2.8e-4 between runs (~1e-3 EPE downstream),
    # while the single-threaded solve is stable and within 2e-6 of the exact solution.
    # The fixtures pin that single-threaded solve.
    lsq_tapped = getattr(sa_mod, "weighted_lsq")

    def lsq_1t(*a, **k):
        nt = torch.get_num_threads()
        torch.set_num_threads(1)
        try:
            return lsq_tapped(*a, **k)
        finally:
            torch.set_num_threads(nt)
    sa_mod.weighted_lsq = lsq_1t
    orig_corr = corr_mod.CorrBlock1D.corr
    corr_mod.CorrBlock1D.corr = staticmethod(tap("corr", orig_corr))
    orig_init = corr_mod.CorrBlock1D.__init__
    orig_call = corr_mod.CorrBlock1D.__call__
    blocks = []

    def init_w(self, fullcorr, *a, **k):
        orig_init(self, fullcorr, *a, **k)
        blocks.append(self)
        if capture_all:
            b = len(blocks) - 1
            for i, p in enumerate(self.corr_pyramid):
                rec[f"pyramid{b}.level{i}"] = _np(p)

    def call_w(self, coords):
        out = orig_call(self, coords)
        b = blocks.index(self)
        n = calls.get(f"lookup{b}", 0)
        calls[f"lookup{b}"] = n + 1
        if capture_all and n < 2:
            rec[f"lookup{b}.{n}.coords"] = _np(coords)
            rec[f"lookup{b}.{n}.out"] = _np(out)
        return out

    corr_mod.CorrBlock1D.__init__ = init_w
    corr_mod.CorrBlock1D.__call__ = call_w
    hooks = []
    if capture_all:
        def fhook(name):
            def h(mod, inp, out):
                if name not in rec:
                    outs = out if isinstance(out, (tuple, list)) else (out,)
                    for i, x in enumerate(outs):
                        if torch.is_tensor(x):
                            rec[f"{name}.out{i}"] = _np(x)
                    ins = inp if isinstance(inp, (tuple, list)) else (inp,)
                    for i, x in enumerate(ins):
                        if torch.is_tensor(x):
                            rec[f"{name}.in{i}"] = _np(x)
            return h
        for name in ["fnet", "hourglass_mono", "classifier_mono", "classifier_monoconf"]:
            hooks.append(getattr(model, name).register_forward_hook(fhook(name)))

        first = {}

        def ub_pre(mod, args, kwargs):
            if "update_block.pre" in first:
                return
            first["update_block.pre"] = 1
            net, inp, corr, corr_mono, flow = args[:5]
            for i, x in enumerate(net):
                rec[f"update_block.0.net_in{i}"] = _np(x)
            for i, lvl in enumerate(inp):
                for j, x in enumerate(lvl):
                    rec[f"update_block.0.inp{i}_{j}"] = _np(x)
            rec["update_block.0.corr"] = _np(corr)
            rec["update_block.0.corr_mono"] = _np(corr_mono)
            rec["update_block.0.flow"] = _np(flow)

        def ub_post(mod, args, kwargs, out):
            if "update_block.post" in first:
                return
            first["update_block.post"] = 1
            net, mask, delta = out
            for i, x in enumerate(net):
                rec[f"update_block.0.net_out{i}"] = _np(x)
            rec["update_block.0.mask"] = _np(mask)
            rec["update_block.0.delta"] = _np(delta)

        hooks.append(model.update_block.register_forward_pre_hook(ub_pre, with_kwargs=True))
        hooks.append(model.update_block.register_forward_hook(ub_post, with_kwargs=True))

    try:
        with torch.no_grad():
            im2 = torch.from_numpy(pair["left"])
            im3 = torch.from_numpy(pair["right"])
            m2 = torch.from_numpy(pair["mono_left"])
            m3 = torch.from_numpy(pair["mono_right"])
            flow_up, _ = model(im2, im3, m2, m3, iters=iters, test_mode=True)
    finally:
        for n in names:
            setattr(sa_mod, n, saved[n])
        corr_mod.CorrBlock1D.corr = staticmethod(orig_corr)
        corr_mod.CorrBlock1D.__init__ = orig_init
        corr_mod.CorrBlock1D.__call__ = orig_call
        for h in hooks:
            h.remove()
    rec["disparity"] = -_np(flow_up)[:, 0]
    return rec


def micro_cases(ut, corr_mod):
    """Per-op known-answer cases with the boundary conditions the reference hits."""
    out = {}
    g = torch.Generator().manual_seed(7)
    # corr with odd widths (pyramid floors at every level), C=256 and C=3
    f2 = torch.randn(2, 256, 3, 37, generator=g)
    f3 = torch.randn(2, 256, 3, 45, generator=g)
    v = corr_mod.CorrBlock1D.corr(f2, f3)
    out.update({"corr.f2": f2, "corr.f3": f3, "corr.out": v})
    blk = corr_mod.CorrBlock1D(v, num_levels=4, radius=4)
    for i, p in enumerate(blk.corr_pyramid):
        out[f"pyr.level{i}"] = p
    # lookup with coordinates inside, at the borders, fractional and far outside
    cx = torch.empty(2, 1, 3, 37).uniform_(-12.0, 57.0, generator=g)
    cx[0, 0, 0, :6] = torch.tensor([0.0, 44.0, -1.0, 45.0, -4.5, 48.999])
    coords = torch.cat([cx, torch.zeros_like(cx)], 1)
    out["lookup.coords"] = coords
    out["lookup.out"] = blk(coords)
    # normals-based mono corr (C=3), masks incl. mde == 1.0 and exact bin edges
    mde = torch.rand(2, 1, 6, 20, generator=g)
    mde[0, 0, 0, :10] = torch.tensor([0.0, 0.125, 0.25, 0.5, 0.875, 1.0, 0.99999, 0.124999, 0.375, 0.625])
    out["masks.mde"] = mde
    out["masks.out"] = ut.generate_masks(mde, N=8).float()
    nrm = ut.estimate_normals(mde, normal_gain=20 / 10)
    out["normals.out"] = nrm
    out["monocorr.out"] = 1.73 * corr_mod.CorrBlock1D.corr(nrm, nrm)
    # soft-argmin / entropy confidence on a peaky and a flat volume
    vol = torch.randn(2, 1, 5, 24, 24, generator=g) * 4.0
    vol[1] = 0.0
    out["sam.vol"] = vol
    out["sam.left"] = ut.estimate_left_disparity(vol)
    out["sam.right"] = ut.estimate_right_disparity(vol)
    out["conf.left"] = ut.estimate_left_confidence(vol)
    out["conf.right"] = ut.estimate_right_confidence(vol)
    # softLRC (W-normalised warping with fractional rows)
    d2 = torch.rand(2, 1, 9, 30, generator=g) * 12 - 1
    d3 = torch.rand(2, 1, 9, 30, generator=g) * 12 - 1
    s2, s3 = ut.softlrc(d2, d3, lrc_th=1.0)
    out.update({"lrc.d2": d2, "lrc.d3": d3, "lrc.s2": s2, "lrc.s3": s3})
    # weighted LSQ with ties and negatives (relu) in the stereo map
    mm = torch.rand(3, 2, 10, 16, generator=g)
    dd = 30 * mm + 4 + torch.randn(3, 2, 10, 16, generator=g)
    dd[0, 0, 0, :20] = -3.0
    dd[1, :, :4] = 7.0
    cc = torch.rand(3, 2, 10, 16, generator=g)
    sc, sh = ut.weighted_lsq(mm, dd, cc)
    out.update({"lsq.mde": mm, "lsq.disp": dd, "lsq.conf": cc, "lsq.scale": sc, "lsq.shift": sh})
    # mirror detector + truncation volume
    dm = torch.rand(2, 1, 4, 16, generator=g) * 10
    ds = torch.rand(2, 1, 4, 16, generator=g) * 10
    cs = torch.rand(2, 1, 4, 16, generator=g)
    cm = torch.rand(2, 1, 4, 16, generator=g)
    mir = ut.handcrafted_mirror_detector(ds, dm, cs, cm, conf_th=0.98)
    tr = ut.truncate_corr_volume_v2(dm, mir, conf_th=None, attenuation_gain=0.9)
    out.update({"mirror.ds": ds, "mirror.dm": dm, "mirror.cs": cs, "mirror.cm": cm, "mirror.out": mir, "trunc.out": tr})
    # convex upsampling
    fl = torch.randn(2, 1, 5, 7, generator=g) * 3
    mk = torch.randn(2, 144, 5, 7, generator=g)
    out.update({"up.flow": fl, "up.mask": mk, "up.out": ut.convex_upflow(fl, mk, n_downsample=2)})
    return {k: _np(v) for k, v in out.items()}


def tiler_cases():
    """The reference tiler (mapreduce_v2/tile_wrapper.py) on a deterministic mock model:
    tile enumeration (incl. duplicate tiles), blend weights and the stitched output."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_tile_wrapper", os.path.join(REF, "mapreduce_v2", "tile_wrapper.py"))
    tw = importlib.util.module_from_spec(spec)
    sys.modules["ref_tile_wrapper"] = tw  # dataclasses resolve their module by name
    spec.loader.exec_module(tw)

    class Mock(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.p = torch.nn.Parameter(torch.zeros(1))

        def forward(self, l, r, ml, mr, iters=1, test_mode=True):
            H, W = l.shape[-2:]
            ramp = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W) / W
            return -(2 * l[:, :1] - r[:, 1:2] + ml * 3 + ramp + H / 100.0), None

    out = {}
    g = torch.Generator().manual_seed(3)
    for i, (H, W, th, tw_, ov) in enumerate([(100, 150, 96, 64, 32), (128, 128, 128, 64, 32), (200, 130, 128, 96, 64),
                                             (96, 96, 128, 128, 32)]):
        l, r = torch.rand(1, 3, H, W, generator=g), torch.rand(1, 3, H, W, generator=g)
        ml, mr = torch.rand(1, 1, H, W, generator=g), torch.rand(1, 1, H, W, generator=g)
        wrap = tw.TileWrapper(Mock(), tile_width=tw_, tile_height=th, overlap=ov)
        tiles = wrap._enumerate_tiles(H, W)
        with torch.no_grad():
            st = wrap(l, r, ml, mr, iters=1, test_mode=True)
        out[f"case{i}.geom"] = np.array([H, W, th, tw_, ov])
        out[f"case{i}.tiles"] = np.array([[t.y_start, t.y_end, t.x_start, t.x_end] for t in tiles])
        out[f"case{i}.weight"] = _np(tw._make_blend_weight(th, tw_, torch.device("cpu")))
        for k, v in (("l", l), ("r", r), ("ml", ml), ("mr", mr), ("out", st)):
            out[f"case{i}.{k}"] = _np(v)
    return out


def mapreduce_cases():
    """The reference's MapReduceInference (mapreduce_v2/tiled_inference.py:25-336) on the
    same mock model: uint8 inputs, bilinear iscale, nearest oscale, post_scale and an
    explicit global-guidance map (the automatic guidance pass needs cv2, absent here).
    The package __init__ imports cv2 (non_lambertian.py), so the three modules are loaded
    as members of a bare package object."""
    import importlib
    pkg = types.ModuleType("ref_mr")
    pkg.__path__ = [os.path.join(REF, "mapreduce_v2")]
    sys.modules["ref_mr"] = pkg
    ti = importlib.import_module("ref_mr.tiled_inference")

    class Mock(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.p = torch.nn.Parameter(torch.zeros(1))

        def forward(self, l, r, ml, mr, iters=1, test_mode=True):
            H, W = l.shape[-2:]
            ramp = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W) / W
            return -(40 * l[:, :1] - 10 * r[:, 1:2] + ml * 3 + ramp + H / 100.0), None

    rng = np.random.default_rng(7)
    out = {}
    cases = [  # H, W, tile_w, tile_h, overlap, iscale, oscale, post_scale, guidance (None / "half" / "full"), weight
        (150, 230, 96, 64, 20, 1.0, 1.0, 1.0, None, 0.3),
        (150, 230, 96, 64, 20, 2.0, 1.0, 1.0, None, 0.3),
        (128, 192, 64, 64, 32, 1.0, 2.0, 1.5, "half", 0.5),
        (128, 192, 64, 64, 32, 1.0, 1.0, 1.0, "full", 0.3),
        (100, 120, 128, 128, 32, 1.0, 1.0, 2.0, "half", 0.5),   # one tile: guidance unused
        (96, 160, 0, 0, 0, 1.0, 1.0, 1.0, None, 0.3),           # square tiles (tile_size 64, overlap 16 -> 32)
    ]
    for i, (H, W, tw_, th, ov, isc, osc, ps, gmode, gw) in enumerate(cases):
        l = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        r = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        ml = torch.from_numpy(rng.random((1, 1, H, W), dtype=np.float32))
        mr = torch.from_numpy(rng.random((1, 1, H, W), dtype=np.float32))
        if tw_:
            inf = ti.MapReduceInference(Mock(), tile_width=tw_, tile_height=th, overlap=ov, guidance_weight=0.2)
        else:
            inf = ti.MapReduceInference(Mock(), tile_size=64, overlap=16, guidance_weight=0.2)
        g = None
        ht, wt = round(H / isc), round(W / isc)
        if gmode == "half":
            g = (rng.random((ht // 2, wt // 2), dtype=np.float32) * 30).astype(np.float32)
        elif gmode == "full":
            g = torch.from_numpy((rng.random((1, 1, ht, wt), dtype=np.float32) * 30).astype(np.float32))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            d = inf.infer(l, r, iscale=isc, oscale=osc, post_scale=ps, mono_pair=(ml, mr), global_guidance=g,
                          guidance_weight=gw, iters=1, test_mode=True)
        out[f"case{i}.geom"] = np.array([H, W, tw_, th, ov], np.int64)
        out[f"case{i}.scales"] = np.array([isc, osc, ps, gw], np.float64)
        out[f"case{i}.l"], out[f"case{i}.r"] = l, r
        out[f"case{i}.ml"], out[f"case{i}.mr"] = _np(ml), _np(mr)
        if g is not None:
            out[f"case{i}.guide"] = g if isinstance(g, np.ndarray) else _np(g)
            out[f"case{i}.guide_is_tensor"] = np.array(not isinstance(g, np.ndarray))
        out[f"case{i}.wrapper"] = np.array([inf.tile_wrapper.tile_width, inf.tile_wrapper.tile_height,
                                            inf.tile_wrapper.overlap])
        out[f"case{i}.out"] = np.asarray(d, np.float32)
    return out


def metrics_cases():
    """losses.guided_metrics (losses.py:273-342) on random disparities with occlusion masks,
    including the all-zero-occlusion branch."""
    tvf = types.ModuleType("torchvision.transforms.functional")
    tvf.gaussian_blur = None
    sys.modules.setdefault("torchvision.transforms", types.ModuleType("torchvision.transforms"))
    sys.modules["torchvision.transforms.functional"] = tvf
    import importlib
    losses = importlib.import_module("losses")
    rng = np.random.default_rng(4)
    out = {}
    for i, occ in enumerate([True, False]):
        gt = (rng.random((1, 1, 40, 60)) * 50).astype(np.float32)
        disp = gt + rng.standard_normal(gt.shape).astype(np.float32) * 3
        valid = (rng.random(gt.shape) > 0.2).astype(np.uint8)
        maskocc = (rng.random(gt.shape) > 0.7).astype(np.uint8) if occ else np.zeros(gt.shape, np.uint8)
        res = losses.guided_metrics(disp, gt, valid, maskocc)
        keys = sorted(k for k in res if k != "errormap")
        out[f"case{i}.disp"], out[f"case{i}.gt"], out[f"case{i}.valid"], out[f"case{i}.occ"] = disp, gt, valid, maskocc
        out[f"case{i}.keys"] = np.array(keys)
        out[f"case{i}.values"] = np.array([float(res[k]) for k in keys], dtype=np.float64)
        out[f"case{i}.errormap"] = res["errormap"].astype(np.float32)
    return out


def odd_size_cases(model):
    """The reference model on sizes that are multiples of 4 but not of 32 — what it accepts
    unpadded (the tiled harness's guidance pass feeds it such sizes, tiled_inference.py:
    199-207): 64x100 (W/4 odd) and 120x168, cropped from one synthetic pair, 4 iterations."""
    base = synth.synthetic_batch(1, 128, 192, 24.0, seed0=5)
    out = {}
    for i, (H, W) in enumerate([(64, 100), (120, 168)]):
        t = [torch.from_numpy(np.ascontiguousarray(base[k][..., :H, :W])) for k in
             ("left", "right", "mono_left", "mono_right")]
        with torch.no_grad():
            flow_up = model(*t, iters=4, test_mode=True)[0]
        for k, v in zip(("left", "right", "mono_left", "mono_right"), t):
            out[f"case{i}.{k}"] = _np(v)
        out[f"case{i}.disparity"] = -_np(flow_up)[:, 0]
    return out


def _pair_record(pair, prefix=""):
    return {f"{prefix}inputs_sha256": np.array(synth.digest([pair[k] for k in ("left", "right", "mono_left",
                                                                               "mono_right")]))}


def wide_case(sa_mod, ut, corr_mod, model):
    """96x1152 (W/4 = 288 > 256, the width class of the booster / kitti / high_memory tile
    presets, tile_presets.py:53-101), 4 iterations: final disparity."""
    pair = synth.synthetic_batch(1, 96, 1152, 64.0, seed0=1)
    rec = run_capture(sa_mod, ut, corr_mod, model, pair, iters=4, capture_all=False)
    return dict(disparity=rec["disparity"].astype(np.float32), **_pair_record(pair))


# (name, H, W, tile_w, tile_h, overlap, D, iters): the presets' tile sides after
# MapReduceInference's rounding (tiled_inference.py:56-69; middlebury overlap 112 -> 128),
# on images sized for two tiles and no duplicate rectangle
TILED_CASES = [
    ("middlebury", 992, 1088, 672, 1120, 128, 256.0, 3),
    ("booster", 672, 1792, 1120, 896, 224, 512.0, 3),
]
ROW_STEP = 4   # stored outputs keep every 4th row (all columns: the tile seams are vertical)


def _single_thread_lsq(sa_mod):
    """Pin the reference's weighted_lsq to the single-threaded (deterministic) solve, as
    run_capture does; returns the restore function."""
    orig = sa_mod.weighted_lsq

    def lsq_1t(*a, **k):
        nt = torch.get_num_threads()
        torch.set_num_threads(1)
        try:
            return orig(*a, **k)
        finally:
            torch.set_num_threads(nt)
    sa_mod.weighted_lsq = lsq_1t
    return lambda: setattr(sa_mod, "weighted_lsq", orig)


def tiled_model_cases(sa_mod, model):
    """The reference TileWrapper (mapreduce_v2/tile_wrapper.py:122-186) driving the
    reference model on seeded weights: a two-tile stitch per preset, plus one full
    Booster-preset tile (896x1120, W/4 = 280) through the model alone.  Outputs keep
    every ROW_STEP-th row to stay small."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_tile_wrapper", os.path.join(REF, "mapreduce_v2", "tile_wrapper.py"))
    tw = importlib.util.module_from_spec(spec)
    sys.modules["ref_tile_wrapper"] = tw
    spec.loader.exec_module(tw)
    restore = _single_thread_lsq(sa_mod)
    out = {"row_step": np.array(ROW_STEP)}
    for i, (name, H, W, tw_, th, ov, D, iters) in enumerate(TILED_CASES):
        pair = synth.synthetic_batch(1, H, W, D, seed0=11 + i)
        t = [torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")]
        wrap = tw.TileWrapper(model, tile_width=tw_, tile_height=th, overlap=ov)
        tiles = wrap._enumerate_tiles(H, W)
        with torch.no_grad():
            st = wrap(*t, iters=iters, test_mode=True)
        out[f"{name}.geom"] = np.array([H, W, tw_, th, ov, iters], np.int64)
        out[f"{name}.D"] = np.array(D)
        out[f"{name}.tiles"] = np.array([[s.y_start, s.y_end, s.x_start, s.x_end] for s in tiles])
        out[f"{name}.out"] = _np(st)[0, 0, ::ROW_STEP].astype(np.float32)
        out.update(_pair_record(pair, f"{name}."))
        print(name, "tiles", len(tiles), "range", float(st.min()), float(st.max()))
    pair = synth.synthetic_batch(1, 896, 1120, 512.0, seed0=13)
    t = [torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")]
    with torch.no_grad():
        d = -model(*t, iters=3, test_mode=True)[0]
    out["booster_tile.geom"] = np.array([896, 1120, 3], np.int64)
    out["booster_tile.out"] = _np(d)[0, 0, ::ROW_STEP].astype(np.float32)
    out.update(_pair_record(pair, "booster_tile."))
    restore()
    return out


# (name, H, W, D, seed): single tiles at the tiled configs' own shapes and iteration count
# (test_mapreduce_v2.py:56 / run_test_contextaware_mapreduce.py:69 run --iters 32): the
# middlebury preset's 1024x672 tile of a 1024-row image (W/16 = 42) and the booster preset's
# 896x1120 tile (W/16 = 70) — GRU levels whose width is not a multiple of 4
TILED32_CASES = [("mb_tile", 1024, 672, 256.0, 31), ("booster_tile", 896, 1120, 512.0, 32)]
# config 3's whole padded image through the reference TileWrapper (middlebury preset): its
# tile grid emits every rectangle twice (y = 0 and y = 992 both clamp to rows 0..1024)
CFG3_IMAGE = (1024, 1408, 672, 1120, 128, 256.0, 33)
TILED32_ROW_STEP = 8


def tiled32_cases(sa_mod, model):
    """The reference model at 32 GRU iterations on one tile of each tiled config, and the
    reference TileWrapper over config 3's whole image (6 tiles, 3 unique rectangles).  Outputs
    keep every TILED32_ROW_STEP-th row."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_tile_wrapper", os.path.join(REF, "mapreduce_v2", "tile_wrapper.py"))
    tw = importlib.util.module_from_spec(spec)
    sys.modules["ref_tile_wrapper"] = tw
    spec.loader.exec_module(tw)
    restore = _single_thread_lsq(sa_mod)
    out = {"row_step": np.array(TILED32_ROW_STEP), "iters": np.array(32)}
    for name, H, W, D, seed in TILED32_CASES:
        pair = synth.synthetic_batch(1, H, W, D, seed0=seed)
        t = [torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")]
        with torch.no_grad():
            d = -model(*t, iters=32, test_mode=True)[0]
        out[f"{name}.geom"] = np.array([H, W, seed], np.int64)
        out[f"{name}.D"] = np.array(D)
        out[f"{name}.out"] = _np(d)[0, 0, ::TILED32_ROW_STEP].astype(np.float32)
        out.update(_pair_record(pair, f"{name}."))
        print(name, "range", float(d.min()), float(d.max()), flush=True)
    H, W, tw_, th, ov, D, seed = CFG3_IMAGE
    pair = synth.synthetic_batch(1, H, W, D, seed0=seed)
    t = [torch.from_numpy(pair[k]) for k in ("left", "right", "mono_left", "mono_right")]
    wrap = tw.TileWrapper(model, tile_width=tw_, tile_height=th, overlap=ov)
    tiles = wrap._enumerate_tiles(H, W)
    with torch.no_grad():
        st = wrap(*t, iters=32, test_mode=True)
    out["cfg3.geom"] = np.array([H, W, tw_, th, ov, seed], np.int64)
    out["cfg3.D"] = np.array(D)
    out["cfg3.tiles"] = np.array([[s.y_start, s.y_end, s.x_start, s.x_end] for s in tiles])
    out["cfg3.out"] = _np(st)[0, 0, ::TILED32_ROW_STEP].astype(np.float32)
    out.update(_pair_record(pair, "cfg3."))
    print("cfg3 tiles", len(tiles), "range", float(st.min()), float(st.max()), flush=True)
    restore()
    return out


def harness_csv_cases():
    """The reference test.py's write_csv_header / write_csv_row (test.py:251-274) on fixed
    metric dicts.  test.py parses argv and builds models at import, so only those two
    functions are taken from its source (ast) and executed; the CSV text is the fixture."""
    import ast
    src = open(os.path.join(REF, "test.py")).read()
    tree = ast.parse(src)
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in ("write_csv_header", "write_csv_row")]
    ns = {}
    exec(compile(ast.Module(body=fns, type_ignores=[]), "reference_test_py", "exec"), ns)
    import io
    rng = np.random.default_rng(9)
    keys = ([f"bad {t}.0" for t in range(1, 9)] + ["avgerr", "rms"] + [f"occ bad {t}.0" for t in range(1, 9)]
            + ["occ avgerr", "occ rms"] + [f"noc bad {t}.0" for t in range(1, 9)] + ["noc avgerr", "noc rms"])
    cases = []
    for j, args in enumerate([
        dict(dataset="middlebury", datapath="dataset/oak_dataset/", monomodel="DAv2", loadmonomodel=None,
             stereomodel="stereoanywhere", loadstereomodel="weights/sceneflow.tar", tries=1, iscale=1.0,
             maxdisp=192, normalize=False),
        dict(dataset="booster", datapath="/data/booster", monomodel="none", loadmonomodel="dav2.pth",
             stereomodel="skip_pred", loadstereomodel="x.tar", tries=3, iscale=2.0, maxdisp=512, normalize=True),
    ]):
        vals = {k: float(np.float32(rng.random() * (1 if "bad" in k else 20))) for k in keys}
        if j == 1:
            vals.update({k: float("nan") for k in keys if k.startswith("occ")})
            vals["occ rms"] = 0.0
        ns_args = types.SimpleNamespace(**args)
        f = io.StringIO()
        ns["write_csv_header"](f, ns_args, vals)
        ns["write_csv_row"](f, ns_args, vals)
        cases.append(dict(args=args, metrics=[[k, vals[k]] for k in keys], text=f.getvalue()))
    return cases


def offload_cases():
    """The reference CPUOffloadWrapper (mapreduce_v2/cpu_offload_wrapper.py:28-83) on CPU
    with a mock stereo model and a mock mono model: mono given, mono computed (offloaded
    to the host and back, or kept), and the error without either."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_offload", os.path.join(REF, "mapreduce_v2",
                                                                              "cpu_offload_wrapper.py"))
    off = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(off)

    class Stereo(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.p = torch.nn.Parameter(torch.ones(1))

        def forward(self, l, r, ml, mr, iters=1, test_mode=True):
            return -(l[:, :1] * 2 - r[:, 2:3] + 3 * ml - mr * 0.5 + iters), None

    class Mono(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.p = torch.nn.Parameter(torch.ones(1))

        def forward(self, l, r):
            return l.mean(1, keepdim=True) * self.p, r.amax(1, keepdim=True)

    g = torch.Generator().manual_seed(21)
    l, r = torch.rand(1, 3, 8, 12, generator=g), torch.rand(1, 3, 8, 12, generator=g)
    ml, mr = torch.rand(1, 1, 8, 12, generator=g), torch.rand(1, 1, 8, 12, generator=g)
    out = {"l": l, "r": r, "ml": ml, "mr": mr}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        with torch.no_grad():
            out["given"] = off.CPUOffloadWrapper(Stereo(), Mono())(l, r, ml, mr, iters=4, test_mode=True)[0]
            out["computed"] = off.CPUOffloadWrapper(Stereo(), Mono())(l, r, iters=2, test_mode=True)[0]
            out["computed_kept"] = off.CPUOffloadWrapper(Stereo(), Mono(), offload_mono=False)(
                l, r, None, None, 3, True)[0]
            try:
                off.CPUOffloadWrapper(Stereo())(l, r)
                msg = ""
            except ValueError as e:
                msg = str(e)
    out = {k: _np(v) for k, v in out.items()}
    out["error_message"] = np.array(msg)
    return out


def _dedupe(rec):
    """Store byte-identical captures once; ``alias.<key>`` names the kept copy."""
    seen, out = {}, {}
    for k in sorted(rec):
        v = np.asarray(rec[k])
        h = (v.dtype.str, v.shape, synth.digest([v]))
        if h in seen and v.nbytes > 64:
            out[f"alias.{k}"] = np.array(seen[h])
        else:
            seen.setdefault(h, k)
            out[k] = v
    return out


# non-published model flags (stereoanywhere.py:141-177): (name, overrides of REF_ARGS, input
# seed); the combinations the reference itself cannot run record the exception type instead.
# addhg2 on seed 3 is ill-conditioned: the reference's own weighted_lsq jumps between two
# solutions (scale -3.76 / -3.72) under 1e-6 noise on its disparity input (its quantile band
# edge), so it runs on seed 4, where 1e-5 noise moves the scale by 1.5e-6.
FLAG_CASES = [
    ("vd1", dict(vol_downsample=1), 3),
    ("aggstereo", dict(use_aggregate_stereo_vol=True), 3),
    ("rawmono", dict(use_aggregate_mono_vol=False), 3),
    ("addhg2", dict(n_additional_hourglass=2), 4),
    ("vd1_rawmono", dict(vol_downsample=1, use_aggregate_mono_vol=False), 3),
    ("vd1_aggstereo", dict(vol_downsample=1, use_aggregate_stereo_vol=True), 3),
]
FLAG_SHAPE = (128, 256, 48.0, 4)   # H, W, max disparity, iterations


def flag_cases(sa_mod, ut, corr_mod):
    """The reference model under each FLAG_CASES configuration (seeded weights, seed 0) on one
    128x256 pair: its parameter names and shapes, and the final disparity or the exception the
    reference raises."""
    H, W, D, iters = FLAG_SHAPE
    out = {}
    for name, over, seed in FLAG_CASES:
        pair = synth.synthetic_batch(1, H, W, D, seed0=seed)
        out.update(_pair_record(pair, f"{name}."))
        out[f"{name}.seed"] = np.array(seed)
        torch.manual_seed(0)
        model = sa_mod.StereoAnywhere(dict(REF_ARGS, **over)).eval()
        synth.load_seeded_weights(model, seed=0)
        out[f"{name}.keys"] = np.array(json.dumps({k: list(v.shape) for k, v in model.state_dict().items()},
                                                  sort_keys=True))
        try:
            # run_capture: the single-threaded least-squares solve the other fixtures pin
            out[f"{name}.disparity"] = run_capture(sa_mod, ut, corr_mod, model, pair, iters,
                                                   capture_all=False)["disparity"].astype(np.float32)
            print(name, "disp range", float(out[f"{name}.disparity"].min()), float(out[f"{name}.disparity"].max()))
        except Exception as e:  # the reference's own failure on this combination
            out[f"{name}.error"] = np.array(type(e).__name__)
            print(name, "raises", type(e).__name__, str(e)[:120])
    return out


DAV2_LAST_BIAS = 0.3


def dav2_cases():
    """Reference Depth Anything V2 (models/depth_anything_v2/dpt.py:168-238) on seeded weights:
    vits ``infer_image`` outputs for a landscape, a portrait (the swapped input size) and a
    square 518 x 518 case (the position grid used as stored), plus every encoder's state-dict
    names and shapes.  cv2 is absent: on this path the reference
    uses it only for the interpolation-method constants its Resize object stores (the resize
    itself is torch's bicubic interpolate, dpt.py:227), so the stub carries those constants."""
    cv2 = sys.modules["cv2"]
    cv2.INTER_NEAREST, cv2.INTER_CUBIC, cv2.INTER_AREA = 0, 2, 3
    tvt = sys.modules.setdefault("torchvision.transforms", types.ModuleType("torchvision.transforms"))
    if not hasattr(tvt, "Compose"):
        tvt.Compose = lambda ts: ts
    from models.depth_anything_v2 import dpt  # noqa
    cfgs = {
        "vits": dict(encoder="vits", features=64, out_channels=[48, 96, 192, 384]),
        "vitb": dict(encoder="vitb", features=128, out_channels=[96, 192, 384, 768]),
        "vitl": dict(encoder="vitl", features=256, out_channels=[256, 512, 1024, 1024]),
        "vitg": dict(encoder="vitg", features=384, out_channels=[1536, 1536, 1536, 1536]),
    }
    out = {}
    init = dpt.DINOv2.__globals__["DinoVisionTransformer"].init_weights
    dpt.DINOv2.__globals__["DinoVisionTransformer"].init_weights = lambda self: None   # names only
    for enc, cfg in cfgs.items():
        m = dpt.DepthAnythingV2(**cfg)
        out[f"keys.{enc}"] = np.array(json.dumps({k: list(v.shape) for k, v in m.state_dict().items()}, sort_keys=True))
        del m
    dpt.DINOv2.__globals__["DinoVisionTransformer"].init_weights = init
    model = dpt.DepthAnythingV2(**cfgs["vits"]).eval()
    synth.load_seeded_weights(model, seed=0)
    # seeded weights drive the head's last conv negative everywhere (its ReLU then outputs 0):
    # its bias is raised so the depth map carries signal
    with torch.no_grad():
        model.depth_head.scratch.output_conv2[2].bias.fill_(DAV2_LAST_BIAS)
    rng = np.random.default_rng(7)
    cases = [("land", (2, 3, 60, 90), 126, 98), ("portrait", (1, 3, 80, 50), 98, 70), ("square", (1, 3, 100, 100), 518, 518)]
    for name, shape, iw, ih in cases:
        raw = rng.random(shape).astype(np.float32)
        with torch.no_grad():
            img, _, (fh, fw) = model.image2tensor(torch.from_numpy(raw.copy()), iw, ih)
            d = model.infer_image(torch.from_numpy(raw.copy()), input_size_width=iw, input_size_height=ih)
        out[f"{name}.raw"] = raw
        out[f"{name}.size"] = np.array([iw, ih, fh, fw], dtype=np.int64)
        out[f"{name}.depth"] = _np(d)
        print("dav2", name, tuple(d.shape), (fh, fw), float(d.min()), float(d.max()), float(d.std()),
              float((d > 0).float().mean()))
    return out


def main(only=None):
    """``python tests/golden/make_golden.py [wide] [tiled] [tiled32] [csv] [offload] [flags] [dav2]`` regenerates
    just the named round-2 fixtures; no argument regenerates everything."""
    torch.set_num_threads(8)
    sa_mod, ut, corr_mod = _load_reference()
    model = build_model(sa_mod)
    if only:
        if "wide" in only:
            np.savez_compressed(os.path.join(HERE, "wide_96x1152_it4.npz"), **wide_case(sa_mod, ut, corr_mod, model))
        if "tiled" in only:
            np.savez_compressed(os.path.join(HERE, "tiled_model.npz"), **tiled_model_cases(sa_mod, model))
        if "tiled32" in only:
            np.savez_compressed(os.path.join(HERE, "tiled32.npz"), **tiled32_cases(sa_mod, model))
        if "csv" in only:
            with open(os.path.join(HERE, "harness_csv.json"), "w") as f:
                json.dump(harness_csv_cases(), f, indent=1)
        if "offload" in only:
            np.savez_compressed(os.path.join(HERE, "offload.npz"), **offload_cases())
        if "flags" in only:
            np.savez_compressed(os.path.join(HERE, "flags.npz"), **flag_cases(sa_mod, ut, corr_mod))
        if "dav2" in only:
            np.savez_compressed(os.path.join(HERE, "dav2.npz"), **dav2_cases())
        return
    np.savez_compressed(os.path.join(HERE, "wide_96x1152_it4.npz"), **wide_case(sa_mod, ut, corr_mod, model))
    np.savez_compressed(os.path.join(HERE, "tiled_model.npz"), **tiled_model_cases(sa_mod, model))
    np.savez_compressed(os.path.join(HERE, "tiled32.npz"), **tiled32_cases(sa_mod, model))
    with open(os.path.join(HERE, "harness_csv.json"), "w") as f:
        json.dump(harness_csv_cases(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "offload.npz"), **offload_cases())
    np.savez_compressed(os.path.join(HERE, "flags.npz"), **flag_cases(sa_mod, ut, corr_mod))
    np.savez_compressed(os.path.join(HERE, "dav2.npz"), **dav2_cases())
    keys = {k: list(v.shape) for k, v in model.state_dict().items()}
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0, sort_keys=True)

    np.savez_compressed(os.path.join(HERE, "micro_ops.npz"), **micro_cases(ut, corr_mod))
    np.savez_compressed(os.path.join(HERE, "tiler.npz"), **tiler_cases())
    np.savez_compressed(os.path.join(HERE, "mapreduce.npz"), **mapreduce_cases())
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), **metrics_cases())
    np.savez_compressed(os.path.join(HERE, "odd_sizes.npz"), **odd_size_cases(model))

    # tiny end-to-end case with every intermediate
    pair = synth.synthetic_batch(1, 64, 128, 24.0, seed0=1)
    rec = run_capture(sa_mod, ut, corr_mod, model, pair, iters=4, capture_all=True)
    rec["inputs_sha256"] = np.array(synth.digest([pair[k] for k in ("left", "right", "mono_left", "mono_right")]))
    for k in ("left", "right", "mono_left", "mono_right"):
        rec[f"input.{k}"] = pair[k]
    np.savez_compressed(os.path.join(HERE, "tiny_64x128_it4.npz"), **_dedupe(rec))

    # config 1: single 256x512 pair, 8 iters — final disparity only
    for (H, W, D, iters, name) in [(256, 512, 64.0, 8, "cfg1_256x512_it8"), (544, 960, 192.0, 22, "cfg2_544x960_it22")]:
        pair = synth.synthetic_batch(1, H, W, D, seed0=1)
        rec = run_capture(sa_mod, ut, corr_mod, model, pair, iters=iters, capture_all=False)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"),
                            disparity=rec["disparity"].astype(np.float32),
                            inputs_sha256=np.array(synth.digest([pair[k] for k in ("left", "right", "mono_left", "mono_right")])))
        print(name, "disp range", rec["disparity"].min(), rec["disparity"].max())


if __name__ == "__main__":
    main(sys.argv[1:])
