"""The test.py harness (reference test.py interface) end to end on the GPU: synthetic
dataset, metrics, CSV; the tiled path through the mapreduce_v2-compatible tiler; and the
reference CLI defaults (use_truncate_vol / use_aggregate_mono_vol off)."""
import csv

import numpy as np
import pytest
import torch

import test as cli
from stereoanywhere_amd import synth, tiler
from stereoanywhere_amd.model import StereoAnywhere

pytestmark = pytest.mark.gpu


def test_cli_synthetic_metrics_and_csv(tmp_path):
    csvp = str(tmp_path / "res.csv")
    mean = cli.main(["--dataset", "synthetic", "--synthetic_size", "120x250", "--synthetic_count", "2", "--iters", "4",
                     "--monomodel", "synthetic", "--use_truncate_vol", "--use_aggregate_mono_vol", "--csv_path", csvp,
                     "--maxdisp", "48", "--outdir", str(tmp_path / "out")])
    assert all(np.isfinite(v) for v in mean.values())
    rows = list(csv.reader(open(csvp)))
    assert rows[0][:4] == ["dataset", "model", "iters", "maxdisp"] and len(rows) == 2


def test_cli_reference_defaults_run():
    mean = cli.main(["--dataset", "synthetic", "--synthetic_size", "64x128", "--synthetic_count", "1", "--iters", "2",
                     "--monomodel", "synthetic", "--maxdisp", "24"])
    assert np.isfinite(mean["avgerr"])


def test_tiled_equals_direct_when_one_tile_and_stitches_otherwise():
    torch.backends.cudnn.benchmark = False
    m = StereoAnywhere(dict(use_truncate_vol=True, use_aggregate_mono_vol=True)).eval()
    synth.load_seeded_weights(m, 0)
    m = m.cuda()
    p = synth.synthetic_batch(1, 160, 320, 40.0, seed0=3)
    t = [torch.from_numpy(p[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
    direct = -m(*t, iters=3, test_mode=True)[0]
    one = tiler.TileWrapper(m, tile_width=320, tile_height=160, overlap=64)(*t, iters=3, test_mode=True)
    assert torch.allclose(one, direct, atol=1e-4)  # image fits one tile: the model runs directly (tile_wrapper.py:151-153)
    tiled = tiler.TileWrapper(m, tile_width=192, tile_height=128, overlap=64)(*t, iters=3, test_mode=True)
    assert tiled.shape == (1, 1, 160, 320) and torch.isfinite(tiled).all()
    # stitched = blend-weighted mean of per-tile forwards: check one pixel covered by a single tile
    tile = tiler.enumerate_tiles(160, 320, 128, 192, 64)[0]
    sub = [x[:, :, tile.y_start:tile.y_end, tile.x_start:tile.x_end] for x in t]
    d = -m(*sub, iters=3, test_mode=True)[0]
    assert torch.allclose(tiled[0, 0, 5, 5], d[0, 0, 5, 5], atol=1e-4)


def test_mapreduce_cli_tiled_with_guidance(tmp_path):
    """test_mapreduce_v2.py (configs 3/5 harness) end to end: 2x3 tiles of 128x192 with the
    automatic low-resolution guidance pass."""
    import test_mapreduce_v2 as mr
    csvp = str(tmp_path / "mr.csv")
    mean = mr.main(["--dataset", "synthetic", "--synthetic_size", "200x320", "--synthetic_count", "1", "--iters", "3",
                    "--monomodel", "synthetic", "--tile_width", "192", "--tile_height", "128", "--overlap", "64",
                    "--use_global_guidance", "--maxdisp", "48", "--csv_path", csvp])
    assert all(np.isfinite(v) for v in mean.values())
    assert len(list(csv.reader(open(csvp)))) == 2
