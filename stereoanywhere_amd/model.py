"""StereoAnywhere on MI355X: the reference model API with the cost-volume hot path on
hand-written HIP kernels (libsa_hip.so) and the dense convolutions on MIOpen fp32.

Drop-in for models/stereoanywhere/stereoanywhere.py:
  * ``StereoAnywhere(args)`` — args is a Namespace or dict; defaults read like the
    reference (stereoanywhere.py:21-50);
  * ``forward(image2, image3, mde2, mde3, iters=12, test_mode=False)`` (95);
    ``test_mode=True`` returns ``(flow_up [B,1,H,W] = -disparity, None)`` (296-297);
  * identical parameter names (state dicts of the reference load with strict=True).

Hot path, one kernel family per row:
  a2+a3  normals + one-hot mono volume records (read by the fused hourglass)  sa_mono_*
  a5+a6  soft-argmin and entropy confidence of the aggregated volumes    sa_softargmin_conf
  a7     softLRC, weighted LSQ (exact quantile band, no host sync)       sa_softlrc, sa_weighted_lsq
  a8+a11 scaled mono, mirror detector, initial coordinates               sa_mono_scale_mirror
  a1+a8+a9 stereo volume x truncation -> pyramid, one fp32-MFMA kernel  sa_corr_volume_pyramid
  a10    stereo + mono pyramid lookups, one launch per iteration         sa_corr_lookup
  a12    GRU gates in the conv epilogues over [h | x | r*h] buffers    sa_conv2d_k3_wino4_multi_gate
  a14    convex upsampling of the final flow                            sa_convex_upsample
Training (test_mode=False) is outside this tier and raises NotImplementedError.
use_truncate_vol / use_aggregate_mono_vol may be off (the reference CLI's store_true
defaults, test.py:94-98).  The non-published flags run on the same kernels with torch glue
around them: vol_downsample > 0 (the masked volume at 1/2^vd as a dense volume, the
classifier outputs trilinearly back to 1/4) and use_aggregate_stereo_vol (the masked stereo
volume through hourglass_stereo + classifier_stereo, times the truncation volume, as the
stereo pyramid); n_additional_hourglass > 1 takes the unfused hourglass.  Combinations the
reference cannot run either raise (tests/golden/flags.npz).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from types import SimpleNamespace

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import encoders, ops
from .blocks import BasicEncoder, BasicMultiUpdateBlock, Hourglass, HourglassIdentity, MultiBasicEncoder
from .corr import HipCorrBlock1D, get_corr_block

_DEFAULTS = dict(
    corr_implementation="hip", n_downsample=2, corr_radius=4, corr_levels=4, n_gru_layers=3,
    encoder_output_dim=128, context_dims=[128] * 3, n_additional_hourglass=0, volume_channels=8, vol_n_masks=8,
    vol_aug_n_masks=4, vol_downsample=0, use_truncate_vol=True, mirror_conf_th=0.98, mirror_attenuation=0.9,
    lrc_th=1, moving_average_decay=0.67, volume_corruption_prob=0.33, normal_gain=10, init_disparity_zero=False,
    use_aggregate_stereo_vol=False, use_aggregate_mono_vol=True, things_to_freeze=["fnet"],
)


def _normalize_pair(a: torch.Tensor, b: torch.Tensor, eps: float = 1e-4):
    """utils.py:56-71 for the C == 1 input path: joint per-(b,c) min/max of the pair."""
    mn = torch.minimum(a.amin(dim=(2, 3), keepdim=True), b.amin(dim=(2, 3), keepdim=True))
    mx = torch.maximum(a.amax(dim=(2, 3), keepdim=True), b.amax(dim=(2, 3), keepdim=True))
    return (a - mn) / (mx - mn + eps), (b - mn) / (mx - mn + eps)



def _drive(gen):
    """Run a generator to its end; its return value."""
    while True:
        try:
            next(gen)
        except StopIteration as e:
            return e.value


@dataclass
class ScheduleOptions:
    """Launch-schedule choices of the MI355X forward.  Every combination computes the same
    function (tests/test_gpu_model.py runs each non-default path against the reference
    fixture); the defaults are the measured-fastest schedule.  Set per instance
    (``model.opts``), e.g. by the A/B scripts under scripts/."""
    # independent 3x3 convs of the update block share one launch (ops.conv2d_k3_multi)
    group_convs: bool = True
    # GRU z/r gates in the F(4x4) conv epilogue where its preconditions hold; False keeps the
    # separate gate kernels
    fuse_gates: bool = True
    # ... and the state update in the r*h conv's epilogue (False: gru_out kernel, r*h conv split
    # over its input channels)
    fuse_out: bool = True
    # mono branch on a second HIP stream beside the encoders (False: one stream)
    mono_stream: bool = True
    # the context encoder on a third stream (2), after the mono branch on the second (1), or on
    # the main stream (0)
    cnet_side: int = 2
    # launches of the update block on F(4x4)'s small blocks (two per CU), by name: "q16" (gru16's
    # r*h conv + the motion conv), "q08" (gru08's + gru32's r*h convs), "zr16", "zr08", "pro32"
    small_launches: frozenset = field(default_factory=frozenset)
    # the encoders' 7x7 stems and stride-2 convs on the direct fp32-MFMA kernel (False: MIOpen)
    direct_conv: bool = True
    # the GRU loop's lookups on disparity-sheared copies of the two pyramids (corr_shear.hip:
    # one load instruction of a wave reads one or two row segments; the row layout spreads
    # it over 64 cache lines); False: the row-layout lookup
    sheared_lookup: bool = True
    # ... when the stereo volume (B x H4 x W4 x W4 floats) is at least shear_min_bytes, written
    # by the two pyramid producers themselves (sheared_producers; stereo: the volume +
    # truncation + pyramid kernel, mono: the pyramid from the classifier output), in rounds of 32
    # pixels so that every sheared row segment is one whole 128-byte line (the row pitch is padded
    # to 32 floats): the stereo producer 203 -> 227 us at cfg2 and 2.68 -> 2.97 ms at the booster
    # batch (round 4's 64 x 64 diagonal tiles, whose segments ended mid-line: 1.27 / 16.3 ms), the
    # lookup 58.7 -> 45.0 us per call in the cfg2 forward (counter bytes 1.2x its bytes model, row
    # layout 2.3x).  sheared_producers=False: a copy pass from the row layout
    # (sa_corr_pyramid_shear, ~190 us per pyramid at cfg2).
    # Memory: a sheared pyramid is ~2x its row-layout one (~3.75x the volume), so the GRU loop
    # holds ~7.5x the volume instead of ~3.75x (e.g. 14 GB for cfg5's 25-tile booster batch); the
    # copy path releases each row pyramid right after its copy (the stereo one before the mono
    # pyramid is built), which bounds it at ~9.4x.  Geometries the sheared kernels do not take
    # (ops.shear_supported: W4 > 511, B * H4 > 65535) keep the row layout.
    sheared_producers: bool = True
    shear_min_bytes: int = 0
    # a GRU level whose width is not a multiple of 4 keeps its planes padded to one (zero
    # columns) and runs on F(4x4) with the gates in the epilogue (False: separate gate kernels and
    # F(2x2) launches for that level)
    pad_ragged: bool = True
    # the GRU loop's batch in this many parts, each on a HIP stream of its own: one part's launch
    # tails and small kernels overlap the other's convs (1: one stream, the whole batch per
    # launch).  B = 4 at 544x960: 82.2 ms/step with 1 part, 79.5 with 2, 86-91 with 3-4 (eager);
    # replayed from a hipGraph (graph.ForwardGraph) 82.3 and 77.5-77.7 (scripts/ab_graph.py)
    loop_parts: int = 2
    # ... part i > 0 starting on the GPU after part i - 1's first half iteration (False: all at
    # once).  Replayed from a hipGraph at the bench config: 74.05-74.22 ms/step against
    # 74.38-74.47 without the offset (three alternating pairs, scripts/ab_graph.py 10 2T 2F ...)
    loop_offset: bool = True
    # the flow head's conv2 (channel 0, the one the model reads) summed in conv1's F(4x4) epilogue
    # and finished with the coordinate update in one small reduction (ops.flow_head_update); False:
    # conv1 written out, then conv2d_k3_narrow and flow_update
    fuse_flow_head: bool = True


class StereoAnywhere(nn.Module):
    def __init__(self, args):
        super().__init__()
        if isinstance(args, dict):
            args = SimpleNamespace(**args)
        for k, v in _DEFAULTS.items():
            if not hasattr(args, k):
                setattr(args, k, v)
        self.args = args
        a = args
        self.cnet = MultiBasicEncoder(output_dim=[a.context_dims, a.context_dims], norm_fn="batch",
                                      downsample=a.n_downsample)
        self.context_zqr_convs = nn.ModuleList(
            [nn.Conv2d(a.context_dims[i], a.context_dims[i] * 3, 3, padding=1) for i in range(a.n_gru_layers)])
        self.fnet = BasicEncoder(output_dim=256, norm_fn="instance", downsample=a.n_downsample)
        self.feature_channels = [1, 1, 1, 1, 1, 1]
        self.hourglass_mono = Hourglass(a.vol_n_masks, a.volume_channels, self.feature_channels)
        self.hourglass_mono_stack = nn.ModuleList([HourglassIdentity()] + [
            Hourglass(a.volume_channels, a.volume_channels, self.feature_channels)
            for _ in range(a.n_additional_hourglass)])
        if a.use_aggregate_stereo_vol:   # stereoanywhere.py:59-65
            self.hourglass_stereo = Hourglass(a.vol_n_masks, a.volume_channels, self.feature_channels)
            self.hourglass_stereo_stack = nn.ModuleList([HourglassIdentity()] + [
                Hourglass(a.volume_channels, a.volume_channels, self.feature_channels)
                for _ in range(a.n_additional_hourglass)])
            self.classifier_stereo = nn.Conv3d(a.volume_channels, 1, 3, 1, 1, bias=False)
        self.classifier_mono = nn.Conv3d(a.volume_channels, 1, 3, 1, 1, bias=False)
        self.classifier_monoconf = nn.Conv3d(a.volume_channels, 1, 3, 1, 1, bias=False)
        self.update_block = BasicMultiUpdateBlock(a.corr_levels, a.corr_radius, a.encoder_output_dim,
                                                  a.context_dims, a.n_downsample)
        self._derived = None
        self._derived_key = None
        # side streams before the update loop (_forward); False runs everything on the
        # caller's stream (bench.py's per-launch event timing)
        self.stream_overlap = True
        self.opts = ScheduleOptions()

    # ------------------------------------------------------------------ weights
    def _split_gru(self, gru, hidden: int):
        wz, wr, wq = gru.convz.weight, gru.convr.weight, gru.convq.weight
        return dict(
            wx=torch.cat([wz[:, hidden:], wr[:, hidden:], wq[:, hidden:]], 0).contiguous(),
            bx=torch.cat([gru.convz.bias, gru.convr.bias, gru.convq.bias], 0).contiguous(),
            whzr=torch.cat([wz[:, :hidden], wr[:, :hidden]], 0).contiguous(),
            wqh=wq[:, :hidden].contiguous(),
            # gates in the conv epilogue: convz | convr over cat(h, x) as the reference has them,
            # and convq's x part
            wzr=torch.cat([wz, wr], 0).contiguous(),
            bzr=torch.cat([gru.convz.bias, gru.convr.bias], 0).contiguous(),
            wqx=wq[:, hidden:].contiguous(),
        )

    def _weights(self):
        """Derived tensors (split GRU kernels, permuted classifier kernels, folded BatchNorm),
        rebuilt when any parameter or buffer is modified or moved."""
        key = tuple((p.data_ptr(), p._version) for p in list(self.parameters()) + list(self.buffers()))
        # (the split kernels' filters are derived only when on)
        key += (self.opts.direct_conv, ops.W4_SPLIT, ops.DIRECT_SPLIT, ops.CONV1X1)
        if self._derived_key != key:
            ub = self.update_block
            hd = self.args.context_dims
            with torch.no_grad():
                self._derived = dict(
                    g08=self._split_gru(ub.gru08, hd[2]), g16=self._split_gru(ub.gru16, hd[1]),
                    g32=self._split_gru(ub.gru32, hd[0]),
                    # reference conv over (H, W1, W2) == conv over (W2, H, W1) with permuted kernel
                    cls_d=self.classifier_mono.weight.permute(0, 1, 4, 2, 3).contiguous(),
                    cls_c=self.classifier_monoconf.weight.permute(0, 1, 4, 2, 3).contiguous(),
                    # convf1 [64,2,7,7] -> [ci][ky][kx][co] for sa_conv2d_small
                    f1=ub.encoder.convf1.weight.permute(1, 2, 3, 0).contiguous(),
                    # encoder._conv has 126 outputs (update.py:78), which drops MIOpen off its
                    # Winograd kernels; two zero filters make it 128 (only 0..125 are read)
                    mot_w=torch.cat([ub.encoder._conv.weight,
                                     ub.encoder._conv.weight.new_zeros((2,) + ub.encoder._conv.weight.shape[1:])]),
                    mot_b=torch.cat([ub.encoder._conv.bias, ub.encoder._conv.bias.new_zeros(2)]),
                )
                enc = ub.encoder
                self._derived.update(
                    # folded eval-BatchNorm affines of the encoders (encoders.py)
                    bn_cnet=encoders.bn_table(self.cnet), bn_fnet=encoders.bn_table(self.fnet),
                    head_b=[(self.cnet.outputs08[0][1].bias, self.cnet.outputs08[1][1].bias),
                            (self.cnet.outputs16[0][1].bias, self.cnet.outputs16[1][1].bias),
                            (self.cnet.outputs32[0].bias, self.cnet.outputs32[1].bias)],
                )
                # Winograd F(2x2,3x3) filters (ops.conv2d_k3) of every eligible 3x3 conv
                d = self._derived
                d["wino"] = encoders.wino_table(self.cnet, self.fnet)
                # eval-BatchNorm norm1 folded into the context encoder's conv1s
                d["fold_cnet"] = encoders.fold_table(self.cnet)
                # the stems and the stride-2 blocks on the direct fp32-MFMA conv (ops.conv_direct)
                # (opts.direct_conv = False leaves them on MIOpen)
                d["direct"] = encoders.direct_table(self.cnet, self.fnet) if self.opts.direct_conv else {}
                for gk in ("g08", "g16", "g32"):
                    g = d[gk]
                    half = g["wqh"].shape[1] // 2
                    g.update(Ux=ops.wino_weights(g["wx"]), Uhzr=ops.wino_weights(g["whzr"]),
                             Uqh=ops.wino_weights(g["wqh"]),
                             Uzr=ops.wino_weights(g["wzr"]), Uqx=ops.wino_weights(g["wqx"]),
                             # the r*h conv split over its input channels (two half-K launches'
                             # worth of blocks; gru_out adds the partial sums)
                             Uqh_k=[ops.wino_weights(g["wqh"][:, :half].contiguous()),
                                    ops.wino_weights(g["wqh"][:, half:].contiguous())])
                d.update(c1_kc=enc.convc1.weight.detach().reshape(enc.convc1.out_channels, -1).t().contiguous(),
                         U_c2=ops.wino_weights(enc.convc2.weight.detach().contiguous()),
                         U_f2=ops.wino_weights(enc.convf2.weight.detach().contiguous()),
                         U_mot=ops.wino_weights(d["mot_w"]),
                         U_fh1=ops.wino_weights(ub.flow_head.conv1.weight.detach().contiguous()),
                         U_mask=ops.wino_weights(ub.mask[0].weight.detach().contiguous()),
                         U_ctx=[ops.wino_weights(c.weight.detach().contiguous()) for c in self.context_zqr_convs],
                         # the 1x1 convs on sa_conv1x1 (None: F.conv2d)
                         c1_fnet=ops.conv1x1_weights(self.fnet.conv2.weight),
                         c1_mask=ops.conv1x1_weights(ub.mask[2].weight))
                cls = torch.cat([self._derived["cls_d"], self._derived["cls_c"]], 0)  # [2,8,3,3,3]
                self._derived["hg"] = self.hourglass_mono.fused_weights(cls)
                if self.args.use_aggregate_stereo_vol:
                    cs = self.classifier_stereo.weight.permute(0, 1, 4, 2, 3).contiguous()
                    self._derived["cls_s"] = cs
                    # the fused classifier pair's second output is unused here
                    self._derived["hg_stereo"] = self.hourglass_stereo.fused_weights(torch.cat([cs, cs], 0))
            self._derived_key = key
        return self._derived

    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    # ------------------------------------------------------------------ forward
    def forward(self, image2, image3, mde2, mde3, iters: int = 12, test_mode: bool = False):
        a = self.args
        if not test_mode:
            raise NotImplementedError("training forward (test_mode=False) is outside the inference tier")
        if a.n_gru_layers != 3 or a.n_downsample != 2:
            raise NotImplementedError("only 3 GRU levels at n_downsample=2 are built")
        if a.vol_downsample > 0 and (a.use_aggregate_stereo_vol or not a.use_aggregate_mono_vol):
            # the reference fails on these combinations too (tests/golden/flags.npz): its
            # full-resolution stereo volume meets the downsampled masks, or its GRU samples the
            # downsampled raw mono volume with full-resolution coordinates
            raise RuntimeError("vol_downsample > 0 needs use_aggregate_mono_vol and no use_aggregate_stereo_vol "
                               "(the reference's volumes stop matching otherwise)")
        get_corr_block(a.corr_implementation)
        if image2.device.type != "cuda":
            raise RuntimeError("StereoAnywhere (MI355X build) runs on the GPU only; move inputs to cuda")
        # the few convs left on MIOpen (1x1 output convs, the mask head's 1x1) on deterministic solvers:
        # at 16 images per launch (configs[3]'s 8 pairs per GPU) the default choice sums in an order
        # that varies from run to run (5e-5 px), which would break bit-stable reruns and graph replays
        cd = torch.backends.cudnn
        with torch.no_grad(), cd.flags(enabled=cd.enabled, benchmark=cd.benchmark, deterministic=True,
                                       allow_tf32=cd.allow_tf32):
            return self._forward(image2, image3, mde2, mde3, iters)

    def _forward(self, image2, image3, mde2, mde3, iters):
        a = self.args
        dw = self._weights()
        B, C, H, W = image2.shape
        if H % 4 or W % 4:
            # the reference fails on these too (its hourglass skip shapes stop matching);
            # callers pad to x32 (test.py:206-213)
            raise RuntimeError(f"H and W must be multiples of 4; got {H}x{W}")
        H4, W4 = H // 4, W // 4
        dev = image2.device
        f32 = torch.float32
        image2, image3 = image2.float(), image3.float()
        if C == 1:
            image2, image3 = _normalize_pair(image2.repeat(1, 3, 1, 1), image3.repeat(1, 3, 1, 1))
        image2 = (image2 * 2 - 1).contiguous()
        image3 = (image3 * 2 - 1).contiguous()
        mde2 = mde2.float().contiguous()
        mde3 = mde3.float().contiguous()

        # ---- mono maps at 1/4 (stereoanywhere.py:109-114): both views in one [B,2,H4,W4] buffer
        mde_lr = torch.empty((B, 2, H4, W4), device=dev, dtype=f32)
        ops.interp(mde2, mde_lr[:, 0:1])
        ops.interp(mde3, mde_lr[:, 1:2])
        m2l = mde_lr[:, 0:1].contiguous()
        m3l = mde_lr[:, 1:2].contiguous()
        gain = W4 / a.normal_gain
        n2 = ops.mono_normals(m2l, gain)
        n3 = ops.mono_normals(m3l, gain)

        # The mono branch (volume -> hourglass -> alignment) reads only the mono maps, so it can
        # run on a second HIP stream beside the encoders, filling their launch tails and
        # HBM-bound passes with the hourglass's compute (opts.mono_stream = False turns it off).  The main stream
        # waits for it before the pyramids; tensors it hands over are recorded on the main
        # stream so the caching allocator does not reuse them early.
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev) if self.opts.mono_stream and self.stream_overlap else None
        if side is not None:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                mono = self._mono_branch(dw, mde2, mde3, mde_lr, m2l, m3l, n2, n3, B, H4, W4)
        # ---- context + feature encoders: 3x3 convs on the HIP Winograd / implicit-GEMM kernels,
        # stems and stride-2 convs on the direct kernel, epilogues fused (encoders.py)
        if self.cnet.training or self.fnet.training:  # batch-statistics BatchNorm: module path
            cl = self.cnet(mde2.repeat(1, 3, 1, 1))
            hid = [torch.tanh(x[0]).contiguous() for x in cl]
            ctx = [conv(torch.relu(x[1])) for x, conv in zip(cl, self.context_zqr_convs)]
            fm = self.fnet(torch.cat([image2, image3], 0))
        else:
            if side is not None and self.opts.cnet_side:
                # the context encoder (it reads only mde2) on a third stream (cnet_side=2)
                # or after the mono branch on the second (1), so the main stream runs the
                # feature encoder alone
                cs = side
                if self.opts.cnet_side == 2:
                    cs = self._side_stream(dev, 1)
                    cs.wait_stream(main)
                with torch.cuda.stream(cs):
                    hid, ctx = self._context(dw, mde2)
                if cs is not side:
                    side.wait_stream(cs)
            else:
                hid, ctx = self._context(dw, mde2)
            fm = encoders.fnet_forward(self.fnet, torch.cat([image2, image3], 0), dw["bn_fnet"], dw["wino"],
                                       dw["direct"], out_w=dw["c1_fnet"])
        fmap2, fmap3 = fm[:B].contiguous(), fm[B:].contiguous()
        if side is not None:
            main.wait_stream(side)
            for t in list(mono) + list(hid) + list(ctx):
                t.record_stream(main)
        else:
            mono = self._mono_branch(dw, mde2, mde3, mde_lr, m2l, m3l, n2, n3, B, H4, W4)
        vol_d, vol_c, sm2, mirror, coords_x = mono
        del mono

        # ---- pyramids
        trunc = (sm2, mirror) if a.use_truncate_vol else (None, None)
        # the sheared lookup for large volumes, where its kernels take the geometry (W4 <= 511,
        # B * H4 <= 65535 image rows, 4 levels of radius 4); the row layout otherwise
        big = (self.opts.sheared_lookup and B * H4 * W4 * W4 * 4 >= self.opts.shear_min_bytes
               and a.corr_levels == 4 and a.corr_radius == 4 and ops.shear_supported(B, H4, W4, W4, a.corr_levels))
        direct = self.opts.sheared_producers and big
        if a.use_aggregate_stereo_vol:
            stereo_blk = self._stereo_aggregate(dw, fmap2, fmap3, mde2, mde3, m2l, m3l, trunc, B, H4, W4)
        else:
            stereo_blk = HipCorrBlock1D.from_features(fmap2, fmap3, a.corr_levels, a.corr_radius, trunc[0], trunc[1],
                                                      float(a.mirror_attenuation), sheared=direct)
        del fmap2, fmap3
        if big and stereo_blk.sheared is None:
            # the sheared copy of the stereo pyramid before the mono pyramid exists, and the row
            # layout released right after it: at most one row pyramid and one sheared copy are
            # live at a time besides the finished copies
            stereo_blk.shear(release=True)
        if a.use_aggregate_mono_vol:
            mono_rows = vol_d.permute(0, 1, 3, 4, 2)  # [B,1,H,W1,W2] view (transposed by the pyramid kernel)
        else:
            # raw mono volume 1.73 * corr(normals) (stereoanywhere.py:136, 210)
            mono_rows = 1.73 * ops.corr_volume(n2, n3)
        mono_blk = HipCorrBlock1D(None, a.corr_levels, a.corr_radius, _shape=(B, H4, W4, W4))
        if direct:
            mono_blk.sheared = ops.pyramid_from_volume_sheared(mono_rows, a.corr_levels)
        if mono_blk.sheared is None:
            mono_blk.pyramid = ops.pyramid_from_volume(mono_rows, a.corr_levels)
        del mono_rows, vol_d, vol_c
        if big and mono_blk.sheared is None:
            # the lookups read disparity-sheared pyramids (coalesced across a wave's pixels); a
            # block whose producer wrote the row layout gets a sheared copy (the row-layout
            # buffer is not read again)
            mono_blk.shear(release=True)
        parts = min(self.opts.loop_parts, B) if self.stream_overlap else 1
        if parts <= 1:
            return _drive(self._iterate(dw, hid, ctx, stereo_blk, mono_blk, coords_x, iters, B, H4, W4))
        return self._iterate_parts(parts, dw, hid, ctx, stereo_blk, mono_blk, coords_x, iters, B, H4, W4)

    def _iterate_parts(self, parts, dw, hid, ctx, stereo_blk, mono_blk, coords_x, iters, B, H4, W4):
        """The GRU loop over batch parts (pairs are independent), each on its own stream; the
        host enqueues them in turn, half an iteration at a time, and part i > 0 starts on the
        GPU once part i - 1 has finished its first half iteration.  The main stream waits for
        every part; the inputs stay referenced until then."""
        dev = coords_x.device
        main = torch.cuda.current_stream(dev)
        bounds = [(B * i // parts, B * (i + 1) // parts) for i in range(parts)]
        rows = H4 * W4

        def blk(b, lo, hi):
            nb = HipCorrBlock1D(None, b.num_levels, b.radius,
                                _pyramid=None if b.pyramid is None else b.pyramid[lo * rows:hi * rows],
                                _shape=(hi - lo, H4, W4, W4))
            if b.sheared is not None:
                nb.sheared = b.sheared[lo * H4:hi * H4]
            return nb
        streams, gens = [], []
        for i, (lo, hi) in enumerate(bounds):
            st = self._loop_stream(dev, i)
            st.wait_stream(main)
            streams.append(st)
            with torch.cuda.stream(st):
                gens.append(self._iterate(dw, [h[lo:hi] for h in hid], [c[lo:hi] for c in ctx],
                                          blk(stereo_blk, lo, hi), blk(mono_blk, lo, hi), coords_x[lo:hi], iters,
                                          hi - lo, H4, W4))
        results = [None] * parts
        first = [None] * parts   # event after each part's first half iteration
        done = [False] * parts
        while not all(done):
            for i in range(parts):
                if done[i] or (i > 0 and first[i - 1] is None):
                    continue
                st = streams[i]
                with torch.cuda.stream(st):
                    if first[i] is None and i > 0 and self.opts.loop_offset:   # before part i's first launch
                        st.wait_event(first[i - 1])
                    try:
                        next(gens[i])
                    except StopIteration as e:
                        results[i], done[i] = e.value, True
                        continue
                    if first[i] is None:
                        first[i] = torch.cuda.Event()
                        first[i].record(st)
        for st, r in zip(streams, results):
            main.wait_stream(st)
            # each part's output was allocated on its loop stream and is read by the cat on
            # main: keep the caching allocator from handing it back to that stream early
            r[0].record_stream(main)
        return torch.cat([r[0] for r in results], 0), None

    def _loop_stream(self, dev, i: int):
        ls = getattr(self, "_loops", None)
        if ls is None or ls[0].device != dev:
            ls = self._loops = []
        while len(ls) <= i:
            ls.append(torch.cuda.Stream(dev))
        return ls[i]

    def _context(self, dw, mde2):
        """Context encoder (eval BatchNorm folded) -> tanh hidden states and the context_zqr
        convs (stereoanywhere.py:116-121)."""
        cl = encoders.cnet_forward(self.cnet, mde2.repeat(1, 3, 1, 1), dw["bn_cnet"], dw["wino"], dw["direct"],
                                   dw["fold_cnet"])
        hid, cs = [], []
        for (h_raw, c_raw), (hb, cb) in zip(cl, dw["head_b"]):
            hid.append(ops.norm_act(h_raw, ops.Affine(t=hb), act_in="tanh", out=h_raw))
            cs.append(ops.norm_act(c_raw, ops.Affine(t=cb), act_in="relu", out=c_raw))
        # the three context_zqr convs ([B,384,..] per level) in one launch
        ctx = ops.conv2d_k3_multi(*[dict(x=c, U=U, bias=conv.bias)
                                    for c, U, conv in zip(cs, dw["U_ctx"], self.context_zqr_convs)])
        return hid, ctx

    def _side_stream(self, dev, i: int = 0):
        ss = getattr(self, "_sides", None)
        if ss is None or ss[0].device != dev:
            ss = self._sides = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        return ss[i]

    def _mono_branch(self, dw, mde2, mde3, mde_lr, m2l, m3l, n2, n3, B, H4, W4):
        """Mono cost volume -> hourglass -> classifiers -> soft-argmin / confidence -> scale-shift
        alignment and mirror detector (stereoanywhere.py:136-205); returns (vol_d, vol_c, scaled
        mono left, mirror map, initial coords_x)."""
        a = self.args
        dev, f32 = mde2.device, torch.float32
        feats_l, feats_r = self._volume_features(mde2, mde3)
        vd = a.vol_downsample

        # ---- mono cost volume -> 3-D hourglass -> classifiers (native [B,C,W2,H,W1] layout)
        # the fused hourglass reads the one-hot masked volume through per-pixel records (its two
        # readers evaluate the cells); the torch path materialises it
        # stack[i] for i < n_additional (stereoanywhere.py:163-164): stack[0] is the identity,
        # so only n_additional >= 2 puts a real hourglass after hourglass_mono
        extra = [self.hourglass_mono_stack[i] for i in range(a.n_additional_hourglass)
                 if not isinstance(self.hourglass_mono_stack[i], HourglassIdentity)]
        if vd > 0:
            # stereoanywhere.py:141-145: the raw volume (trilinear) and the masks (nearest) at
            # 1/2^vd, masked as a dense volume (the downsampled cells are no longer a product of
            # per-pixel terms)
            vol = (1.73 * ops.corr_volume(n2, n3)).view(B, 1, H4, W4, W4)
            masked = self._masked_dense(vol, m2l, m3l, vd)
            fuse = not extra and a.vol_n_masks == 8 and self.hourglass_mono.fusable(masked, feats_l)
        else:
            # the one-hot records only where the fused hourglass will read them; the torch path
            # gets the materialised volume
            shape = SimpleNamespace(shape=(B, a.vol_n_masks, W4, H4, W4))
            fuse = not extra and a.vol_n_masks == 8 and self.hourglass_mono.fusable(shape, feats_l)
            masked = (ops.OneHotVolume(n2, n3, m2l, m3l, a.vol_n_masks, 1.73) if fuse
                      else ops.mono_masked_volume(n2, n3, m2l, m3l, a.vol_n_masks, 1.73))
        if fuse:
            vol_d, vol_c = self.hourglass_mono(masked, feats_l, feats_r, fused=dw["hg"])
        else:
            agg = self.hourglass_mono(masked, feats_l, feats_r)
            for hg in extra:
                agg = hg(agg, feats_l, feats_r)
            vol_d = F.conv3d(agg, dw["cls_d"], padding=1)  # [B,1,W2,H,W1]
            vol_c = F.conv3d(agg, dw["cls_c"], padding=1)
            del agg
        del masked
        if vd > 0:
            # back to the 1/4 grid (stereoanywhere.py:170-172); the native axis order (W2, H, W1)
            # of the same per-axis trilinear interpolation
            up = dict(size=(W4, H4, W4), mode="trilinear", align_corners=True)
            vol_d, vol_c = F.interpolate(vol_d, **up), F.interpolate(vol_c, **up)
        # (b, h, j, k) -> native [B, ., W2, H, W1] layout; vol_d/vol_c may be channel views
        strides = (vol_d.stride(0), W4, 1, H4 * W4)
        disp_lr, conf_lr = ops.softargmin_conf(vol_d, vol_c, strides, (B, H4, W4, W4))

        # ---- scale/shift alignment, mirror detector, truncation inputs
        confx = ops.softlrc_joint(disp_lr, conf_lr, float(a.lrc_th))          # fuzzy_and(conf, softlrc)
        scale, shift = ops.weighted_lsq(mde_lr, disp_lr, confx)
        sm2, sm3, mirror, coords_x = ops.mono_scale_mirror(mde_lr, scale, shift, disp_lr, confx,
                                                           float(a.lrc_th), float(a.mirror_conf_th))
        if a.init_disparity_zero:
            coords_x = torch.arange(W4, device=dev, dtype=f32).expand(B, 1, H4, W4).contiguous()
        return vol_d, vol_c, sm2, mirror, coords_x

    def _volume_features(self, mde2, mde3):
        """The hourglasses' guidance pyramids fmde2 / fmde3 (stereoanywhere.py:111-112, 122-123):
        the mono maps at the volume's resolution (1/2^vol_downsample), then at 1/2^i for
        i = n_downsample .. 5."""
        a = self.args

        def resized(m, i):   # F.interpolate(scale_factor=2^-i)'s output size: floor(size * 2^-i)
            B, C, H, W = m.shape
            return torch.empty((B, C, H >> i, W >> i), device=m.device, dtype=torch.float32)

        out = []
        for m in (mde2, mde3):
            m = m.contiguous()
            if a.vol_downsample > 0:
                m = ops.interp(m, resized(m, a.vol_downsample))
            levels = [resized(m, i) for i in range(a.n_downsample, len(self.feature_channels))]
            # the levels as jobs of one resample launch each (align_corners bilinear, sa_resample_multi)
            for k in range(0, len(levels), 4):
                ops.resample_multi(*[("interp", m, o, None, None) for o in levels[k:k + 4]])
            out.append(levels)
        return out

    def _masked_dense(self, vol, m2l, m3l, vd: int) -> torch.Tensor:
        """vol [B,1,H,W1,W2] x the depth-bin masks of the 1/4-res mono maps (generate_masks,
        utils.py:48-54: bin n holds n/N <= m < (n+1)/N), both at 1/2^vd when vd > 0
        (stereoanywhere.py:141-145, 147, 161) -> the hourglass's [B, N, W2, H, W1] layout."""
        N = self.args.vol_n_masks

        def masks(m):
            n = torch.arange(N, device=m.device, dtype=m.dtype).view(1, N, 1, 1)
            return ((m < (n + 1) / N) & (m >= n / N)).to(torch.float16)
        ml, mr = masks(m2l), masks(m3l)
        if vd > 0:
            vol = F.interpolate(vol, scale_factor=1 / 2 ** vd, mode="trilinear", align_corners=True)
            ml = F.interpolate(ml, scale_factor=1 / 2 ** vd, mode="nearest")
            mr = F.interpolate(mr, scale_factor=1 / 2 ** vd, mode="nearest")
        masked = vol * ml.unsqueeze(4) * mr.unsqueeze(3)            # [B, N, H, W1, W2]
        return masked.permute(0, 1, 4, 2, 3).contiguous()

    def _stereo_aggregate(self, dw, fmap2, fmap3, mde2, mde3, m2l, m3l, trunc, B, H4, W4):
        """use_aggregate_stereo_vol (stereoanywhere.py:147-157, 201-205, 253-255): the masked
        stereo volume through hourglass_stereo and classifier_stereo, times the truncation
        volume, as the GRU's stereo pyramid (the coarse stereo disparities the reference also
        forms there are not used by the test-mode forward)."""
        a = self.args
        vol = ops.corr_volume(fmap2, fmap3).view(B, 1, H4, W4, W4)
        masked = self._masked_dense(vol, m2l, m3l, 0)
        del vol
        feats_l, feats_r = self._volume_features(mde2, mde3)
        extra = [self.hourglass_stereo_stack[i] for i in range(a.n_additional_hourglass)
                 if not isinstance(self.hourglass_stereo_stack[i], HourglassIdentity)]
        if not extra and a.vol_n_masks == 8 and self.hourglass_stereo.fusable(masked, feats_l):
            vol_s = self.hourglass_stereo(masked, feats_l, feats_r, fused=dw["hg_stereo"])[0]
        else:
            agg = self.hourglass_stereo(masked, feats_l, feats_r)
            for hg in extra:
                agg = hg(agg, feats_l, feats_r)
            vol_s = F.conv3d(agg, dw["cls_s"], padding=1)
            del agg
        del masked
        rows = vol_s.permute(0, 1, 3, 4, 2)       # [B, 1, H, W1, W2] view
        if trunc[0] is not None:
            # truncate_corr_volume_v2 (utils.py:216-238), conf_th=None
            d, m = trunc[0].view(B, 1, H4, W4, 1), trunc[1].view(B, 1, H4, W4, 1)
            j = torch.arange(W4, device=d.device, dtype=d.dtype).view(1, 1, 1, W4, 1)
            k = torch.arange(W4, device=d.device, dtype=d.dtype).view(1, 1, 1, 1, W4)
            att = float(a.mirror_attenuation)
            T = 1 * (1 - m) + m * (torch.sigmoid((j - d) - k) * (1 - att) + att)
            rows = T * rows
        return HipCorrBlock1D(None, a.corr_levels, a.corr_radius,
                              _pyramid=ops.pyramid_from_volume(rows.contiguous(), a.corr_levels),
                              _shape=(B, H4, W4, W4))

    def _iterate(self, dw, hid, ctx, stereo_blk, mono_blk, coords_x, iters, B, H4, W4):
        """The GRU loop as a generator: it yields twice per iteration (after gru16 and at the
        end) so that batch parts on separate streams can be enqueued in turn (_iterate_parts);
        its return value is (flow_up, None)."""
        ub = self.update_block
        enc = ub.encoder
        dev = coords_x.device
        f32 = torch.float32
        h08, h16, h32 = hid
        H8, W8 = h16.shape[2:]
        H16, W16 = h32.shape[2:]
        c1 = torch.empty((2 * B, enc.convc1.out_channels, H4, W4), device=dev, dtype=f32)  # convc1(lookups)
        motin = torch.empty((B, 192, H4, W4), device=dev, dtype=f32)  # [convc2 stereo | mono | convf2]
        flow = torch.empty((B, 2, H4, W4), device=dev, dtype=f32)
        # x08 = [motion(126) | flow(2) | interp(h16)], x16 = [pool(h08) | interp(h32)], x32 = [pool(h16)]
        xdims = {"08": 256, "16": 256, "32": 128}
        shapes = {"08": (H4, W4), "16": (H8, W8), "32": (H16, W16)}
        lvl_of = {"08": 0, "16": 1, "32": 2}
        hd = h08.shape[1]
        o = self.opts
        # GRU gates in the F(4x4) conv epilogues, per level.  A level whose width is not a
        # multiple of 4 (e.g. W/16 = 42 or 70 at the middlebury / booster tile presets) keeps
        # its state in PITCHED planes, rows padded to a multiple of 4 with zero columns
        # (opts.pad_ragged), which F(4x4) reads as the right zero padding and keeps zero in its
        # outputs; without it that level keeps the separate gate kernels and F(2x2) launches of
        # its own (ops.conv2d_k3_multi splits a mixed group).
        f4 = o.fuse_gates and ops.gate_f4_ok()
        # (not the 1/4 level: its planes are also read and written by the lookup, motion and
        # flow kernels, which take dense planes only)
        fused = {k: f4 and (s[1] % 4 == 0 or (o.pad_ragged and k != "08")) for k, s in shapes.items()}
        # row pitch of each level's GRU planes (its width unless padded) and the conv width
        pitch = {k: (s[1] + 3) // 4 * 4 if fused[k] else s[1] for k, s in shapes.items()}
        wid = {k: s[1] if pitch[k] != s[1] else None for k, s in shapes.items()}
        # (a padded level always updates its state in the r*h conv's epilogue: the gate kernels
        # take dense planes)
        fuse_out = {k: fused[k] and (o.fuse_out or wid[k] is not None) for k in shapes}
        hxr, xq, rh, xs = {}, {}, {}, {}
        ctxp = list(ctx)
        for k, h in zip(("08", "16", "32"), hid):
            if fused[k]:
                padded = wid[k] is not None
                alloc = torch.zeros if padded else torch.empty
                Hk, Wk = shapes[k]
                # one buffer per level, [h | x | r*h]: the z/r conv reads cat(h, x) and the r*h
                # conv reads r*h as channel views of it (no torch.cat)
                hxr[k] = alloc((B, 2 * hd + xdims[k], Hk, pitch[k]), device=dev, dtype=f32)
                hxr[k][:, :hd, :, :Wk].copy_(h)
                xs[k] = hxr[k][:, hd:hd + xdims[k]]
                rh[k] = hxr[k][:, hd + xdims[k]:]
                # convq's x part lands in channels 2*hd.. of a [B, 3*hd] buffer: gru_out reads it there
                xq[k] = alloc((B, 3 * hd, Hk, pitch[k]), device=dev, dtype=f32)
                if padded:   # the context planes cz | cr | cq of the level, pitched once per forward
                    c = ctx[lvl_of[k]]
                    cp = torch.zeros((B, c.shape[1], Hk, pitch[k]), device=dev, dtype=f32)
                    cp[..., :Wk].copy_(c)
                    ctxp[lvl_of[k]] = cp
            else:
                xs[k] = torch.empty((B, xdims[k], *shapes[k]), device=dev, dtype=f32)
                rh[k] = torch.empty_like(h)
        ctx = ctxp
        h08, h16, h32 = (hxr[k][:, :hd] if fused[k] else h for k, h in zip(("08", "16", "32"), hid))
        x08, x16, x32 = xs["08"], xs["16"], xs["32"]
        hs = {"08": h08, "16": h16, "32": h32}
        z = {k: (torch.zeros if wid[k] is not None else torch.empty)(h.shape, device=dev, dtype=f32)
             for k, h in hs.items()}
        cz = [c[:, 0:128] for c in ctx]
        cr = [c[:, 128:256] for c in ctx]
        cq = [c[:, 256:384] for c in ctx]
        lvl = lvl_of

        def conv_group(*probs, name=None):
            """Independent 3x3 convs in one launch (opts.group_convs = False: one launch each)."""
            if o.group_convs:
                return ops.conv2d_k3_multi(*probs, small_blocks=name in o.small_launches)
            return [ops.conv2d_k3_multi(p, small_blocks=name in o.small_launches)[0] for p in probs]

        def gate_x_h(key, x, h):
            g = dw["g" + key]
            if fused[key]:
                # convz | convr over cat(h, x) (+ bias) with z = sigmoid(. + cz) and r*h = sigmoid(. + cr) * h
                # in the epilogue (update.py:24-25); convq's x part (bias added in gru_out)
                hx = hxr[key][:, :hd + xdims[key]]
                return [dict(x=hx, U=g["Uzr"], bias=g["bzr"], out=z[key], width=wid[key],
                             gate=dict(mode=1, ctx=ctx[lvl[key]], h=h, out2=rh[key])),
                        dict(x=x, U=g["Uqx"], out=xq[key][:, 2 * hd:], width=wid[key])]
            # x and h halves of convz/convr/convq; bias added in the gate kernels
            return [dict(x=x, U=g["Ux"]), dict(x=h, U=g["Uhzr"])]

        def gru_zr(level, key, h, xc, hzr):
            if not fused[key]:   # else done in the conv epilogue
                ops.gru_zr(xc, hzr, cz[level], cr[level], h, z[key], rh[key], bx=dw["g" + key]["bx"])

        def gru_out(level, key, h, xc, qh, qh2=None):
            ops.gru_out(xq[key] if fused[key] else xc, qh, cq[level], z[key], h, bx=dw["g" + key]["bx"], qh2=qh2)

        def qh_split(key):
            """r*h conv of one GRU as two half-Cin problems (more, shorter blocks: the launch's
            last round of blocks costs less)."""
            r, Uk = rh[key], dw["g" + key]["Uqh_k"]
            c = r.shape[1] // 2
            return [dict(x=r[:, :c], U=Uk[0]), dict(x=r[:, c:], U=Uk[1])]

        def q_probs(key, split):
            """convq's r*h part: with the state update h = (1 - z) h + z tanh(. + x part + cq) in
            its epilogue (one problem, in place on h), else plain problem(s) (split over Cin when
            ``split``) whose sums q_finish hands to gru_out."""
            if fuse_out[key]:
                g = dw["g" + key]
                return [dict(x=rh[key], U=g["Uqh"], bias=g["bx"][2 * hd:], out=hs[key], width=wid[key],
                             gate=dict(mode=2, ctx=cq[lvl[key]], h=hs[key], z=z[key], add=xq[key][:, 2 * hd:]))]
            return qh_split(key) if split else [dict(x=rh[key], U=dw["g" + key]["Uqh"])]

        def q_finish(level, key, xc, res):
            if not fuse_out[key]:
                gru_out(level, key, hs[key], xc, *res)

        ops.flow_update(coords_x, None, flow, x08[:, 126:128])
        flow_up = None
        c1v = c1.view(B, 2, c1.shape[1], H4, W4)
        # update.py:164-197 runs, per iteration, gru32 -> gru16 -> motion encoder -> gru08 -> flow
        # head.  gru32 of iteration k+1 reads only h16 and h32 as they are after gru16 of
        # iteration k, so it runs one iteration early, in the launches of gru08's convs; the
        # motion encoder reads neither GRU state, so its convs share gru16's launches.  Every op
        # is deterministic and reads the same inputs as in the reference order: the result is
        # identical, with fewer and fuller conv launches.
        def pool(src, ks, dst, kd):
            ops.pool2x(src, dst, width=wid[ks], out_width=wid[kd])

        pool(h16, "16", x32, "32")
        xc32, hzr32 = conv_group(*gate_x_h("32", x32, h32), name="pro32")
        gru_zr(2, "32", h32, xc32, hzr32)
        q_finish(2, "32", xc32, conv_group(*q_probs("32", False), name="pro32"))
        for it in range(iters):
            last = it == iters - 1
            # lookup of both pyramids + convc1 + ReLU in one kernel (sample 2b: stereo, 2b+1: mono)
            stereo_blk.lookup_conv1x1_into(coords_x, dw["c1_kc"], enc.convc1.bias, c1, other=mono_blk)
            # (the flow's vertical channel is identically zero, written so by flow_update: convf1
            # over channel 0 alone adds the same products, without the 49 zero taps)
            fl = ops.conv2d_small(flow[:, :1], dw["f1"], enc.convf1.bias, 64, 7, relu=True)
            # pool2x(h08) and interp(h32) into gru16's input, one launch
            ops.resample_multi(("pool", h08, x16[:, :128], wid["08"], wid["16"]),
                               ("interp", h32, x16[:, 128:], wid["32"], wid["16"]))
            # gru16's x/h convs + the motion encoder's 3x3 convs (bias + ReLU in the epilogue,
            # written straight into the motion conv's input cat(convc2(stereo), convc2(mono),
            # convf2(convf1(flow))))
            mconv = [dict(x=c1v[:, v], U=dw["U_c2"], bias=enc.convc2.bias, relu=True,
                          out=motin[:, 64 * v:64 * v + 64]) for v in range(2)]
            mconv.append(dict(x=fl, U=dw["U_f2"], bias=enc.convf2.bias, relu=True, out=motin[:, 128:192]))
            xc16, hzr16 = conv_group(*gate_x_h("16", x16, h16), *mconv, name="zr16")[:2]
            gru_zr(1, "16", h16, xc16, hzr16)
            # gru16's r*h conv + the motion conv (_conv: 126 outputs, padded to 128, into
            # x08[:, :128]; channels 126-127 (the flow) are rewritten right after)
            qp = q_probs("16", False)
            res = conv_group(*qp, dict(x=motin, U=dw["U_mot"], bias=dw["mot_b"], relu=True, out=x08[:, :128]),
                             name="q16")
            q_finish(1, "16", xc16, res[:len(qp)])
            yield   # half an iteration (the batch-parts schedule interleaves here)
            # the flow planes of x08 (after the motion conv wrote its padding channels there),
            # interp(h16) into gru08's input and (not last) pool2x(h16) into gru32's, one launch
            ops.resample_multi(("flow_x", coords_x, x08[:, 126:128], None, None),
                               ("interp", h16, x08[:, 128:], wid["16"], wid["08"]),
                               *([] if last else [("pool", h16, x32, wid["16"], wid["32"])]))
            # gru08's x/h convs (+ gru32's of the next iteration), then the r*h convs
            probs = gate_x_h("08", x08, h08)
            if not last:
                probs += gate_x_h("32", x32, h32)
            res = conv_group(*probs, name="zr08")
            xc08, hzr08 = res[:2]
            gru_zr(0, "08", h08, xc08, hzr08)
            qp = q_probs("08", True)
            probs = list(qp)
            if not last:
                xc32, hzr32 = res[2:]
                gru_zr(2, "32", h32, xc32, hzr32)
                probs += q_probs("32", True)
            qh = conv_group(*probs, name="q08")
            q_finish(0, "08", xc08, qh[:len(qp)])
            if not last:
                q_finish(2, "32", xc32, qh[len(qp):])
            # flow head + coordinate update (update.py:98-110, stereoanywhere.py:283-285); fused: conv1's
            # epilogue sums conv2's channel-0 taps, so conv1's 256-channel output is never written
            if not (o.fuse_flow_head and ops.flow_head_update(h08, dw["U_fh1"], ub.flow_head.conv1.bias,
                                                              ub.flow_head.conv2.weight, ub.flow_head.conv2.bias,
                                                              coords_x, flow)):
                f1 = ops.conv2d_k3(h08, dw["U_fh1"], ub.flow_head.conv1.bias, relu=True)
                delta = ops.conv2d_k3_narrow(f1, ub.flow_head.conv2.weight, ub.flow_head.conv2.bias)
                ops.flow_update(coords_x, delta[:, 0:1], flow, None)
            if it == iters - 1:
                # mask head (update.py:185-191): 3x3 conv + bias + ReLU on the Winograd kernel,
                # then the 1x1 conv; x 0.25 as the reference scales it
                m1 = ops.conv2d_k3(h08, dw["U_mask"], ub.mask[0].bias, relu=True)
                if dw["c1_mask"] is not None:
                    mask = ops.conv1x1(m1, dw["c1_mask"], ub.mask[2].out_channels, ub.mask[2].bias, 0.25)
                else:
                    mask = F.conv2d(m1, ub.mask[2].weight, ub.mask[2].bias).mul_(0.25)
                flow_up = ops.convex_upsample(flow[:, 0:1].contiguous(), mask, 2 ** self.args.n_downsample)
            yield
        return flow_up, None
