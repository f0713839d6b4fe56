"""The tiled configs at their own iteration count (32: test_mapreduce_v2.py:56,
run_test_contextaware_mapreduce.py:69) against the REFERENCE model / TileWrapper
(tests/golden/make_golden.py tiled32_cases, seeded weights):

* one middlebury-preset tile, 1024x672 (GRU widths 168 / 84 / 42: the 1/16 level has
  W % 4 != 0, so its planes are padded to 44 columns and it runs on F(4x4) with the gates in
  the epilogue, ScheduleOptions.pad_ragged);
* one booster-preset tile, 896x1120 (280 / 140 / 70);
* config 3's whole padded image (1024x1408) through the tiler: 6 tiles, 3 unique rectangles,
  each run once and accumulated twice;
* config 5's whole padded Booster image (3008x4128, 25 tiles) under CPUOffloadWrapper: finite,
  and its single-coverage corner equals the per-tile forward.

Fixtures keep every 8th row.  Gate: EPE < 1e-3."""
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
    return load_fixture("tiled32.npz")


def _inputs(fix, prefix, H, W, D, seed):
    pair = synth.synthetic_batch(1, H, W, D, seed0=seed)
    got = synth.digest([pair[k] for k in ("left", "right", "mono_left", "mono_right")])
    assert got == str(fix[f"{prefix}.inputs_sha256"]), "synthetic inputs differ from the fixture's"
    return [torch.from_numpy(pair[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("name", ["mb_tile", "booster_tile"])
def test_tile_32_iterations_vs_reference(model, fix, monkeypatch, name, split):
    """split: the F(4x4) and direct convs on the f16 hi/lo split kernels (ops.W4_SPLIT,
    ops.DIRECT_SPLIT) or all on fp32 MFMA products."""
    from stereoanywhere_amd import ops
    monkeypatch.setattr(ops, "W4_SPLIT", split)
    monkeypatch.setattr(ops, "DIRECT_SPLIT", split)
    H, W, seed = (int(v) for v in fix[f"{name}.geom"])
    x = _inputs(fix, name, H, W, float(fix[f"{name}.D"]), seed)
    # the 1/16 GRU level is ragged (W/16 = 42 or 70): padded planes on F(4x4)
    assert (W // 16) % 4 != 0 and (W // 4) % 4 == 0 and (W // 8) % 4 == 0
    with torch.no_grad():
        d = -model(*x, iters=32, test_mode=True)[0]
    got = d[0, 0, ::int(fix["row_step"])].cpu().numpy()
    e = epe(got, fix[f"{name}.out"])
    print(name, "split" if split else "fp32", "EPE", e, "max", float(np.abs(got - fix[f"{name}.out"]).max()))
    assert np.isfinite(got).all()
    assert e < 1e-3


@pytest.mark.parametrize("option", ["fuse_gates", "pad_ragged"])
def test_tile_32_iterations_fallback_schedule(model, fix, option):
    """The same booster tile with the gates kept out of the conv epilogues at every level
    (ScheduleOptions.fuse_gates = False), or only at the ragged 1/16 level (pad_ragged = False:
    F(2x2) and the separate gate kernels there, split out of the shared launches)."""
    H, W, seed = (int(v) for v in fix["booster_tile.geom"])
    x = _inputs(fix, "booster_tile", H, W, 512.0, seed)
    saved = getattr(model.opts, option)
    setattr(model.opts, option, False)
    try:
        with torch.no_grad():
            d = -model(*x, iters=32, test_mode=True)[0]
    finally:
        setattr(model.opts, option, saved)
    got = d[0, 0, ::int(fix["row_step"])].cpu().numpy()
    e = epe(got, fix["booster_tile.out"])
    print("booster tile (unfused gates) EPE", e)
    assert e < 1e-3


def test_cfg3_image_deduplicated_tiles_vs_reference(model, fix):
    H, W, tw, th, ov, seed = (int(v) for v in fix["cfg3.geom"])
    x = _inputs(fix, "cfg3", H, W, float(fix["cfg3.D"]), seed)
    p = tiler.get_preset("middlebury")
    assert (tw, th, ov) == tiler.tiling_for(p.tile_width, p.tile_height, p.overlap)
    wrap = tiler.TileWrapper(model, tile_width=tw, tile_height=th, overlap=ov, batch_tiles=True)
    tiles = wrap._enumerate_tiles(H, W)
    assert [[t.y_start, t.y_end, t.x_start, t.x_end] for t in tiles] == fix["cfg3.tiles"].tolist()
    with torch.no_grad():
        st = wrap(*x, iters=32, test_mode=True)
    assert wrap.last_tile_counts == (6, 3)
    got = st[0, 0, ::int(fix["row_step"])].cpu().numpy()
    e = epe(got, fix["cfg3.out"])
    print("cfg3 image EPE", e, "max", float(np.abs(got - fix["cfg3.out"]).max()))
    assert e < 1e-3


def test_cfg5_full_booster_image():
    """Config 5's whole image: 3008x4128 (3008x4112 padded to x32), booster preset -> 25
    tiles of 896x1120, 32 iterations, CPUOffloadWrapper, tiles batched.  Finite, and rows
    0..672 x columns 0..896 (covered by the first tile alone) equal that tile's own forward."""
    m = StereoAnywhere(dict(PUBLISHED)).eval()
    synth.load_seeded_weights(m, 0)
    m = m.cuda()
    H, W = 3008, 4128
    pair = synth.synthetic_batch(1, H, W, 512.0, seed0=1)
    x = [torch.from_numpy(pair[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
    wrap = tiler.from_preset(m, "booster", batch_tiles=True)
    tiles = wrap._enumerate_tiles(H, W)
    assert len(tiles) == 25 and len(set(tiles)) == 25
    assert {(t.height, t.width) for t in tiles} == {(896, 1120)}
    with torch.no_grad():
        st = CPUOffloadWrapper(wrap)(*x, iters=32, test_mode=True)
        assert tuple(st.shape) == (1, 1, H, W)
        assert bool(torch.isfinite(st).all())
        t0 = tiles[0]
        one = -m(*[v[:, :, t0.y_start:t0.y_end, t0.x_start:t0.x_end] for v in x], iters=32, test_mode=True)[0]
    a = st[0, 0, :672, :896].cpu().numpy().astype(np.float64)
    b = one[0, 0, :672, :896].cpu().numpy().astype(np.float64)
    print("cfg5 corner vs tile forward: EPE", np.abs(a - b).mean(), "max", np.abs(a - b).max())
    # the batched forward of 25 tiles against one tile alone: the same per-tile arithmetic except
    # for library convs whose algorithm may depend on the batch (measured: 1.05e-5 mean, 8.4e-5 max)
    assert np.abs(a - b).mean() < 5e-5 and np.abs(a - b).max() < 1e-3
