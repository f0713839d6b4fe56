"""The test.py harness (reference test.py interface) end to end on the GPU: the per-sample
disparity equals the model's direct forward on the padded inputs (which is pinned to the
reference in test_gpu_model.py), the CSV is the reference's layout, --tries aggregates;
the tiled harness through the mapreduce_v2-compatible tiler; the reference CLI defaults
(use_truncate_vol / use_aggregate_mono_vol off)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import test as cli
from stereoanywhere_amd import data, harness, synth, tiler
from stereoanywhere_amd.model import StereoAnywhere

pytestmark = pytest.mark.gpu


def test_cli_disparity_is_the_model_forward_and_csv(tmp_path):
    csvp = str(tmp_path / "res.csv")
    args = ["--dataset", "synthetic", "--synthetic_size", "120x250", "--synthetic_count", "2", "--iters", "4",
            "--monomodel", "synthetic", "--use_truncate_vol", "--use_aggregate_mono_vol", "--csv_path", csvp,
            "--maxdisp", "48", "--outdir", str(tmp_path / "out"), "--tries", "2"]
    mean = cli.main(args)
    # all 30 columns: the synthetic pairs carry an occlusion mask (data.SyntheticPairs)
    assert all(np.isfinite(mean[k]) for k in harness.METRIC_ORDER), {k: mean[k] for k in harness.METRIC_ORDER}
    lines = open(csvp).read().splitlines()
    assert len(lines) == 2 and lines[0].split(",")[10:] == [k.upper() for k in harness.METRIC_ORDER]
    assert lines[1].split(",")[:10] == ["synthetic", "dataset/oak_dataset/", "synthetic", "None", "stereoanywhere",
                                        "None", "2", "1.0", "48", "False"]
    # sample 1's written disparity == -model(padded inputs), unpadded (test.py:204-230)
    m = StereoAnywhere(dict(use_truncate_vol=True, use_aggregate_mono_vol=True)).eval()
    synth.load_seeded_weights(m, 0)
    m = m.cuda()
    s = data.SyntheticPairs(2, 120, 250, 48.0)[1]
    x = [torch.from_numpy(s[k])[None].cuda() for k in ("im2", "im3", "im2_mono", "im3_mono")]
    lo, hi = torch.minimum(x[2].min(), x[3].min()), torch.maximum(x[2].max(), x[3].max())
    x[2], x[3] = (x[2] - lo) / (hi - lo), (x[3] - lo) / (hi - lo)
    pad = tiler.pad32(120, 250)
    with torch.no_grad():
        d = -m(*[F.pad(t, pad, mode="replicate") for t in x], iters=4, test_mode=True)[0][0, 0]
    d = d[pad[2]:d.shape[0] - pad[3], pad[0]:d.shape[1] - pad[1]].cpu().numpy()
    written = data.read_pfm(str(tmp_path / "out" / "synthetic1_disp.pfm"))
    assert written.shape == (120, 250)
    assert np.abs(written - d).mean() < 1e-5


def test_cli_reference_defaults_run():
    mean = cli.main(["--dataset", "synthetic", "--synthetic_size", "64x128", "--synthetic_count", "1", "--iters", "2",
                     "--monomodel", "synthetic", "--maxdisp", "24"])
    assert np.isfinite(mean["avgerr"])


def test_cli_skip_pred():
    """--stereomodel skip_pred: zero prediction, no network (test.py:127-128, 219-228)."""
    mean = cli.main(["--dataset", "synthetic", "--synthetic_size", "64x128", "--synthetic_count", "2",
                     "--stereomodel", "skip_pred", "--monomodel", "none", "--maxdisp", "24"])
    s = [data.SyntheticPairs(2, 64, 128, 24.0)[i]["gt"] for i in range(2)]
    np.testing.assert_allclose(mean["avgerr"], np.mean([np.float32(g.mean()) for g in s]), rtol=1e-6)


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
    # all 30 columns: the synthetic pairs carry an occlusion mask (data.SyntheticPairs)
    assert all(np.isfinite(mean[k]) for k in harness.METRIC_ORDER), {k: mean[k] for k in harness.METRIC_ORDER}
    assert len(open(csvp).read().splitlines()) == 2
