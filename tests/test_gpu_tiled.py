"""Configs 3 and 5 on the GPU: the mapreduce_v2-compatible tiler driving the MI355X model at
the reference presets' tile sizes, against fixtures the REFERENCE TileWrapper + reference
model produced on the same seeded weights and inputs (tests/golden/make_golden.py
tiled_model_cases; reduced iterations), and the full harness at the configs' workloads.

* middlebury preset: 672x1120 tiles, overlap 112 -> 128 (tiled_inference.py:66-69), a
  992x1088 image = two 992x672 tiles (W/4 = 168);
* booster preset: 1120x896 tiles, overlap 224, a 672x1792 image = two 672x1120 tiles, and
  one full 896x1120 tile (W/4 = 280 > 256) through the model alone.
Fixtures keep every 4th row (all columns: the seams are vertical).  Gate: EPE < 1e-3."""
import numpy as np
import pytest
import torch

from fixtures_util import epe, load_fixture
from stereoanywhere_amd import synth, tiler
from stereoanywhere_amd.model import StereoAnywhere
from stereoanywhere_amd.offload import CPUOffloadWrapper

pytestmark = pytest.mark.gpu
PUBLISHED = dict(use_truncate_vol=True, use_aggregate_mono_vol=True)


@pytest.fixture(scope="module")
def model():
    m = StereoAnywhere(dict(PUBLISHED)).eval()
    synth.load_seeded_weights(m, 0)
    return m.cuda()


@pytest.fixture(scope="module")
def fix():
    return load_fixture("tiled_model.npz")


def _inputs(fix, prefix, H, W, D, seed):
    pair = synth.synthetic_batch(1, H, W, D, seed0=seed)
    got = synth.digest([pair[k] for k in ("left", "right", "mono_left", "mono_right")])
    assert got == str(fix[f"{prefix}.inputs_sha256"]), "synthetic inputs differ from the fixture's"
    return [torch.from_numpy(pair[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]


@pytest.mark.parametrize("i,name", [(0, "middlebury"), (1, "booster")])
@pytest.mark.parametrize("offload", [False, True])
def test_two_tile_stitch_vs_reference(model, fix, i, name, offload):
    H, W, tw, th, ov, iters = (int(v) for v in fix[f"{name}.geom"])
    p = tiler.get_preset(name)
    assert (tw, th, ov) == tiler.tiling_for(p.tile_width, p.tile_height, p.overlap)
    x = _inputs(fix, name, H, W, float(fix[f"{name}.D"]), 11 + i)
    wrap = tiler.TileWrapper(model, tile_width=tw, tile_height=th, overlap=ov)
    tiles = wrap._enumerate_tiles(H, W)
    assert [[t.y_start, t.y_end, t.x_start, t.x_end] for t in tiles] == fix[f"{name}.tiles"].tolist()
    runner = CPUOffloadWrapper(wrap) if offload else wrap
    with torch.no_grad():
        st = runner(*x, iters=iters, test_mode=True)
    got = st[0, 0, ::int(fix["row_step"])].cpu().numpy()
    e = epe(got, fix[f"{name}.out"])
    print(name, "stitch EPE", e, "max", float(np.abs(got - fix[f"{name}.out"]).max()))
    assert e < 1e-3


def test_booster_tile_vs_reference(model, fix):
    H, W, iters = (int(v) for v in fix["booster_tile.geom"])
    x = _inputs(fix, "booster_tile", H, W, 512.0, 13)
    with torch.no_grad():
        d = -model(*x, iters=iters, test_mode=True)[0]
    got = d[0, 0, ::int(fix["row_step"])].cpu().numpy()
    e = epe(got, fix["booster_tile.out"])
    print("booster tile EPE", e, "max", float(np.abs(got - fix["booster_tile.out"]).max()))
    assert e < 1e-3


def test_cfg3_harness_middlebury_preset():
    """Config 3's workload through test_mapreduce_v2.main: a Middlebury-H-sized synthetic
    pair (1000x1400 -> padded 1024x1408: three 1024x672 tiles), middlebury preset, 32
    iterations, end to end (the tiler and the model it drives are pinned above)."""
    import test_mapreduce_v2 as mr
    mean = mr.main(["--dataset", "synthetic", "--synthetic_size", "1000x1400", "--synthetic_count", "1",
                    "--maxdisp", "256", "--iters", "32", "--monomodel", "synthetic", "--tile_preset", "middlebury",
                    "--use_truncate_vol", "--use_aggregate_mono_vol"])
    assert np.isfinite(mean["avgerr"]) and np.isfinite(mean["bad 2.0"])


def test_cfg5_harness_booster_preset_with_offload(tmp_path):
    """Config 5's tiling: booster preset (1120x896 tiles, overlap 224) under the
    CPUOffloadWrapper on a 1792x2464 synthetic pair (3x3 = 9 tiles), 32 iterations; the
    harness output equals the wrapper-free tiler on the same uint8 inputs."""
    import test_mapreduce_v2 as mr
    from stereoanywhere_amd import data
    args = ["--dataset", "synthetic", "--synthetic_size", "1792x2464", "--synthetic_count", "1", "--maxdisp", "512",
            "--iters", "32", "--monomodel", "synthetic", "--tile_preset", "booster", "--use_truncate_vol",
            "--use_aggregate_mono_vol", "--outdir", str(tmp_path)]
    mean = mr.main(args + ["--cpu_offload"])
    assert np.isfinite(mean["avgerr"])
    a = data.read_pfm(str(tmp_path / "synthetic0_disp.pfm"))
    mr.main(args)
    b = data.read_pfm(str(tmp_path / "synthetic0_disp.pfm"))
    assert a.shape == (1792, 2464) and np.isfinite(a).all()
    assert epe(a, b) < 1e-5


class _GpuMock(torch.nn.Module):
    """A deterministic per-tile 'model' on the GPU (negated disparity, position- and size-dependent)."""

    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.zeros(1, device="cuda"))
        self.calls = []

    def forward(self, l, r, ml, mr, iters=1, test_mode=True):
        self.calls.append(tuple(l.shape))
        H, W = l.shape[-2:]
        ramp = torch.arange(W, dtype=torch.float32, device=l.device).view(1, 1, 1, W) / W
        return -(40 * l[:, :1] - 10 * r[:, 1:2] + ml * 3 - mr + ramp + H / 100.0), None


@pytest.mark.parametrize("H,W,th,tw,ov", [(300, 500, 160, 224, 64), (256, 416, 256, 224, 96), (200, 260, 96, 128, 32)])
def test_tile_gather_and_stitch_equal_torch_path(monkeypatch, H, W, th, tw, ov):
    """The GPU gather (sa_tile_gather_pad: cat + replicate pad) and stitch (sa_tile_stitch) equal
    the torch path bit for bit: the padded batch the model sees and the stitched map, including
    geometries whose enumeration lists a rectangle twice and ragged tiles (non-multiples of 32)."""
    g = torch.Generator(device="cpu").manual_seed(H + W)
    imgs = [torch.rand(1, c, H, W, generator=g).cuda() for c in (3, 3, 1, 1)]
    out = {}
    seen = {}
    for hip in (True, False):
        if not hip:
            monkeypatch.setattr(tiler, "_hip_tiles", lambda *ts: False)
        m = _GpuMock()
        tw_ = tiler.TileWrapper(m, tile_width=tw, tile_height=th, overlap=ov, batch_tiles=True)
        out[hip] = tw_(*imgs, iters=1, test_mode=True)
        seen[hip] = m.calls
    assert seen[True] == seen[False]
    assert torch.equal(out[True], out[False]), float((out[True] - out[False]).abs().max())
