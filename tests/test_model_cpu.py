"""Host-side model checks (no GPU): parameter names are the reference's, seeded weights
load strictly, and the product refuses to run on the CPU (no fallback path)."""
import json
import os

import pytest
import torch

from fixtures_util import GOLDEN
from stereoanywhere_amd import synth
from stereoanywhere_amd.model import StereoAnywhere

PUBLISHED = dict(use_truncate_vol=True, use_aggregate_mono_vol=True, vol_n_masks=8, n_additional_hourglass=0,
                 vol_downsample=0, mirror_conf_th=0.98, mirror_attenuation=0.9)


def test_state_dict_names_match_reference():
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))
    m = StereoAnywhere(dict(PUBLISHED))
    ours = {k: list(v.shape) for k, v in m.state_dict().items()}
    assert ours == ref


@pytest.mark.parametrize("name,over", [("aggstereo", dict(use_aggregate_stereo_vol=True)),
                                       ("addhg2", dict(n_additional_hourglass=2)), ("vd1", dict(vol_downsample=1))])
def test_state_dict_names_match_reference_under_flags(name, over):
    """The non-published flags' extra modules (hourglass_stereo, its stack, classifier_stereo,
    additional hourglasses) carry the reference's names and shapes (tests/golden/flags.npz)."""
    import numpy as np
    fix = np.load(os.path.join(GOLDEN, "flags.npz"))
    ref = json.loads(str(fix[f"{name}.keys"]))
    m = StereoAnywhere(dict(PUBLISHED, **over))
    assert {k: list(v.shape) for k, v in m.state_dict().items()} == ref


def test_reference_checkpoint_layout_loads_strict():
    m = StereoAnywhere(dict(PUBLISHED))
    sd = {k: torch.from_numpy(v) for k, v in synth.seeded_state_dict(
        {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()}
    # DataParallel-wrapped checkpoints carry a 'module.' prefix (test.py:142-152)
    wrapped = {"state_dict": {"module." + k: v for k, v in sd.items()}}
    from stereoanywhere_amd.checkpoint import load_reference_checkpoint
    load_reference_checkpoint(m, wrapped)
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k]), k


def test_cpu_inputs_are_refused():
    m = StereoAnywhere(dict(PUBLISHED)).eval()
    x = torch.zeros(1, 3, 64, 128)
    with pytest.raises(RuntimeError, match="GPU"):
        m(x, x, x[:, :1], x[:, :1], iters=1, test_mode=True)


def test_training_forward_not_built():
    m = StereoAnywhere(dict(PUBLISHED))
    x = torch.zeros(1, 3, 64, 128)
    with pytest.raises(NotImplementedError):
        m(x, x, x[:, :1], x[:, :1], iters=1, test_mode=False)


def test_unknown_corr_implementation_raises_like_reference():
    m = StereoAnywhere(dict(PUBLISHED, corr_implementation="alt"))
    x = torch.zeros(1, 3, 64, 128)
    with pytest.raises(NotImplementedError):
        m(x, x, x[:, :1], x[:, :1], iters=1, test_mode=True)
