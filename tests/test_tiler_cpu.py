"""The tiler against the reference's own TileWrapper (tests/golden/tiler.npz, made by
running mapreduce_v2/tile_wrapper.py on a deterministic mock model): tile grid incl.
duplicate tiles, blend weights, pad/unpad, negation and the stitched result."""
import numpy as np
import pytest
import torch

from fixtures_util import load_fixture
from stereoanywhere_amd import tiler


class Mock(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.zeros(1))   # TileWrapper.device reads the model's parameters

    def forward(self, l, r, ml, mr, iters=1, test_mode=True):
        H, W = l.shape[-2:]
        ramp = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W) / W
        return -(2 * l[:, :1] - r[:, 1:2] + ml * 3 + ramp + H / 100.0), None


@pytest.fixture(scope="module")
def fix():
    return load_fixture("tiler.npz")


@pytest.mark.parametrize("i", range(4))
def test_tiles_weights_and_stitch_match_reference(fix, i):
    H, W, th, tw, ov = [int(v) for v in fix[f"case{i}.geom"]]
    tiles = tiler.enumerate_tiles(H, W, th, tw, ov)
    assert [[t.y_start, t.y_end, t.x_start, t.x_end] for t in tiles] == fix[f"case{i}.tiles"].tolist()
    np.testing.assert_allclose(tiler.blend_weight(th, tw, "cpu").numpy(), fix[f"case{i}.weight"], atol=0)
    t = {k: torch.from_numpy(fix[f"case{i}.{k}"]) for k in ("l", "r", "ml", "mr")}
    for batch in (False, True):
        wrap = tiler.TileWrapper(Mock(), tile_width=tw, tile_height=th, overlap=ov, batch_tiles=batch)
        out = wrap(t["l"], t["r"], t["ml"], t["mr"], iters=1, test_mode=True)
        # cases 0-2 enumerate duplicate rectangles (10/8, 8/3, 20/9 tiles/unique): each unique one
        # runs once and is added with its multiplicity, and the stitch still equals the reference's
        assert wrap.last_tile_counts == (len(tiles), len(set(tiles)))
        np.testing.assert_allclose(out.numpy(), fix[f"case{i}.out"], atol=1e-6)


def test_duplicate_tiles_are_kept():
    # 128-px image, 128-px tile, 64 overlap -> the same rectangle twice
    # (and the last column twice: x = 192 and 256 both clamp to [172, 300))
    tiles = tiler.enumerate_tiles(128, 300, 128, 128, 64)
    assert len(tiles) == 10 and len(set(tiles)) == 4
    assert {(t.y_start, t.y_end) for t in tiles} == {(0, 128)}


def test_preset_rounding():
    # middlebury preset: 672x1120, overlap 112 -> 128 (tiled_inference.py:66-69)
    assert tiler.tiling_for(672, 1120, 112) == (672, 1120, 128)
    assert tiler.tiling_for(1120, 896, 224) == (1120, 896, 224)
    assert tiler.tiling_for(500, 300, 0) == (512, 320, 0)
