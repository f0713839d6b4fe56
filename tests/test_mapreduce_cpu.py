"""MapReduceInference and the TileWrapper API against the reference's own mapreduce_v2
(tests/golden/mapreduce.npz, made by running tiled_inference.py on a mock model): uint8
inputs, bilinear iscale, nearest oscale, post_scale, explicit global guidance (resized to
the input, blended per tile; unused when the image fits one tile), square / rectangular
tile rounding.  The automatic guidance pass calls cv2 (absent in this image), so its area
down-sampler is checked against its definition here — parity unpinned against cv2."""
import numpy as np
import pytest
import torch

from fixtures_util import load_fixture
from stereoanywhere_amd import tiler


class Mock(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.zeros(1))

    def forward(self, l, r, ml, mr, iters=1, test_mode=True):
        H, W = l.shape[-2:]
        ramp = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W) / W
        return -(40 * l[:, :1] - 10 * r[:, 1:2] + ml * 3 + ramp + H / 100.0), None


@pytest.fixture(scope="module")
def fix():
    return load_fixture("mapreduce.npz")


@pytest.mark.parametrize("i", range(6))
def test_mapreduce_infer_matches_reference(fix, i):
    H, W, tw, th, ov = [int(v) for v in fix[f"case{i}.geom"]]
    isc, osc, ps, gw = [float(v) for v in fix[f"case{i}.scales"]]
    if tw:
        inf = tiler.MapReduceInference(Mock(), tile_width=tw, tile_height=th, overlap=ov, guidance_weight=0.2)
    else:
        inf = tiler.MapReduceInference(Mock(), tile_size=64, overlap=16, guidance_weight=0.2)
    w = inf.tile_wrapper
    assert [w.tile_width, w.tile_height, w.overlap] == fix[f"case{i}.wrapper"].tolist()
    g = fix.get(f"case{i}.guide")
    if g is not None and bool(fix[f"case{i}.guide_is_tensor"]):
        g = torch.from_numpy(g)
    ml, mr = torch.from_numpy(fix[f"case{i}.ml"]), torch.from_numpy(fix[f"case{i}.mr"])
    d = inf.infer(fix[f"case{i}.l"], fix[f"case{i}.r"], iscale=isc, oscale=osc, post_scale=ps, mono_pair=(ml, mr),
                  global_guidance=g, guidance_weight=gw, iters=1, test_mode=True)
    assert d.shape == fix[f"case{i}.out"].shape
    np.testing.assert_allclose(d, fix[f"case{i}.out"], atol=2e-5, rtol=1e-6)


def test_tilewrapper_constructor_matches_reference():
    m = Mock()
    sq = tiler.TileWrapper(m, 384)                       # square, positional tile_size
    assert (sq.tile_width, sq.tile_height, sq.use_rectangular) == (384, 384, False)
    rect = tiler.TileWrapper(m, None, 96, 64, 32)
    assert (rect.tile_width, rect.tile_height, rect.overlap, rect.use_rectangular) == (96, 64, 32, True)
    assert rect.device == torch.device("cpu")
    with pytest.raises(ValueError):
        tiler.TileWrapper(m)                             # neither square nor rectangular
    with pytest.raises(ValueError):
        tiler.TileWrapper(m, tile_size=64, overlap=-1)
    with pytest.raises(ValueError):
        tiler.TileWrapper(m, tile_width=96, tile_height=64, overlap=64)
    assert tiler.TileWrapper(m, 512).overlap == 256      # default overlap 256 < 512 is fine ...
    with pytest.raises(ValueError):
        tiler.TileWrapper(m, 256)                        # ... 256 is not


def test_tilewrapper_input_validation():
    w = tiler.TileWrapper(Mock(), tile_width=64, tile_height=64, overlap=32)
    l = torch.rand(1, 3, 100, 100)
    with pytest.raises(ValueError):
        w(l, torch.rand(1, 3, 100, 90))
    with pytest.raises(ValueError):
        w(l, l, torch.rand(1, 1, 90, 100), None)
    with pytest.raises(ValueError):
        w(torch.rand(2, 3, 100, 100), torch.rand(2, 3, 100, 100))


def test_guidance_blend_formula():
    d = torch.tensor([[1.0, 2.0], [3.0, 10.0]])
    g = torch.tensor([[1.0, 4.0], [3.0, 2.0]])
    out = tiler.guidance_blend(d, g, 0.5)
    diff = (d - g).abs()
    conf = 1 - diff / (diff.max() + 1e-6)
    ref = (1 - 0.5 * conf) * d + 0.5 * conf * g
    torch.testing.assert_close(out, ref, atol=0, rtol=0)
    assert out[0, 0] == 1.0 and abs(float(out[1, 1]) - 10.0) < 1e-5   # max-diff pixel keeps its value


def test_uint8_truncation():
    t = torch.tensor([[[[-0.5, 0.0, 0.999, 1.0, 2.0, 0.5019]]]]).expand(1, 3, 1, 6)
    img = tiler.to_uint8_image(t)
    assert img.dtype == np.uint8 and img.shape == (1, 6, 3)
    assert img[0, :, 0].tolist() == [0, 0, 254, 255, 255, 127]   # truncation, not rounding


def test_area_resize_definition():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (10, 14, 3), dtype=np.uint8)
    # integer factor: block means, half rounded up
    out = tiler.resize_area_u8(img, 7, 5)
    blocks = img.reshape(5, 2, 7, 2, 3).astype(np.int64).sum(axis=(1, 3))
    assert np.array_equal(out, ((blocks + 2) // 4).astype(np.uint8))
    # fractional factor: each output is a convex combination of the source cells it covers
    out = tiler.resize_area_u8(img, 5, 4)
    assert out.shape == (4, 5, 3)
    x = img.astype(np.float64)
    s_y, s_x = 10 / 4, 14 / 5
    ref00 = x[:2, :2].sum(0).sum(0) + 0.5 * x[2, :2].sum(0) + 0.8 * x[:2, 2].sum(0) + 0.4 * x[2, 2]
    np.testing.assert_allclose(out[0, 0], np.rint(ref00 / (s_y * s_x)), atol=0)
    with pytest.raises(ValueError):
        tiler.resize_area_u8(img, 20, 5)


def test_auto_guidance_pass_runs_untiled_at_low_resolution():
    calls = []

    class Spy(Mock):
        def forward(self, l, r, ml, mr, iters=1, test_mode=True):
            calls.append((tuple(l.shape[-2:]), iters))
            return super().forward(l, r, ml, mr, iters, test_mode)

    rng = np.random.default_rng(1)
    l = rng.integers(0, 256, (128, 192, 3), dtype=np.uint8)
    r = rng.integers(0, 256, (128, 192, 3), dtype=np.uint8)
    mono = (torch.rand(1, 1, 128, 192), torch.rand(1, 1, 128, 192))
    inf = tiler.MapReduceInference(Spy(), tile_width=64, tile_height=64, overlap=32, use_global_guidance=True)
    inf.infer(l, r, mono_pair=mono, iters=1, test_mode=True)
    assert calls[0] == ((64, 96), 32)            # low-res pass, iters hard-coded to 32
    n = len(calls)
    inf.infer(l, r, mono_pair=mono, iters=1, test_mode=True)
    assert len(calls) == 2 * n - 1               # guidance cached by image content
    g = inf._compute_global_guidance(l, r, mono, torch.device("cpu"), torch.float32)
    assert g.shape == (128, 192) and g.dtype == np.float32


def test_mapreduce_harness_procedure():
    """test_mapreduce_v2.py run_mapreduce (178-301) on the CPU with a spy model: the model sees
    padded uint8-quantised images and jointly normalised mono maps; the output is unpadded to
    the ground truth's shape."""
    import test_mapreduce_v2 as cli
    from stereoanywhere_amd import data

    seen = []

    class Spy(Mock):
        def forward(self, l, r, ml, mr, iters=1, test_mode=True):
            seen.append((l.clone(), ml.clone(), mr.clone(), iters, test_mode))
            return super().forward(l, r, ml, mr, iters, test_mode)

    args = cli.build_parser().parse_args(["--dataset", "synthetic", "--tile_width", "64", "--tile_height", "64",
                                          "--overlap", "32", "--iters", "3", "--monomodel", "synthetic"])
    assert cli.apply_preset(args)
    inf = cli.build_inferencer(Spy(), args)
    assert (inf.tile_wrapper.tile_width, inf.tile_wrapper.tile_height, inf.tile_wrapper.overlap) == (64, 64, 32)
    sample = data.SyntheticPairs(1, 90, 150, 24.0)[0]
    res = cli.run_mapreduce(sample, args, torch.device("cpu"), inf)
    assert res["disp"].shape == (1, 90, 150) and np.isfinite(res["avgerr"])
    l, ml, mr, iters, tm = seen[0]
    assert iters == 3 and tm is True and tuple(l.shape[-2:]) == (64, 64)
    q = l * 255
    assert torch.allclose(q, q.round(), atol=1e-4)                    # uint8 grid
    mono = torch.cat([torch.from_numpy(sample["im2_mono"]), torch.from_numpy(sample["im3_mono"])])
    lo, hi = mono.min(), mono.max()
    assert float(torch.stack([s[1] for s in seen]).min()) >= 0.0
    assert float(torch.stack([s[1] for s in seen]).max()) <= float((sample["im2_mono"].max() - lo) / (hi - lo)) + 1e-6


def test_presets_by_name_and_dataset():
    import test_mapreduce_v2 as cli
    args = cli.build_parser().parse_args(["--dataset", "booster", "--tile_preset", "auto"])
    assert cli.apply_preset(args) and (args.tile_width, args.tile_height, args.overlap) == (1120, 896, 224)
    args = cli.build_parser().parse_args(["--tile_preset", "middlebury", "--overlap", "64"])
    assert cli.apply_preset(args) and (args.tile_width, args.tile_height, args.overlap) == (672, 1120, 64)
    assert tiler.get_preset_for_dataset("kitti2015").name == "kitti"
    assert tiler.get_preset_for_dataset("eth3d").name == "default"
    with pytest.raises(ValueError):
        tiler.get_preset("nope")
