"""sa_feature_gates (csrc/gate2d.hip): the hourglass's DoubleFeatureAtt branches
(submodule.py:113-140) against the torch modules they replace, float64, and in batches of jobs
of different sizes and channel counts."""
import numpy as np
import pytest
import torch

from stereoanywhere_amd import ops
from stereoanywhere_amd.blocks import DoubleFeatureAtt

pytestmark = pytest.mark.gpu


def _att(cv_chan, seed):
    torch.manual_seed(seed)
    att = DoubleFeatureAtt(cv_chan, 1).cuda().eval()
    with torch.no_grad():   # non-trivial biases / scales
        for p in att.parameters():
            p.mul_(1.5).add_(0.05)
    return att


@pytest.mark.parametrize("shape", [(2, 34, 60), (4, 68, 120), (1, 136, 240), (3, 17, 29)])
def test_feature_gates_match_torch_modules(shape):
    B, H, W = shape
    atts = [_att(c, c + H) for c in (16, 32, 8)]
    feats = [torch.rand(B, 1, H, W, device="cuda") * 3 - 1 for _ in atts]
    jobs = []
    for att, f in zip(atts, feats):
        jobs += [(f, ops.feature_gate_weights(att.feat_att_left)), (f.flip(-1).contiguous(),
                                                                     ops.feature_gate_weights(att.feat_att_right))]
    outs = ops.feature_gates(jobs)
    with torch.no_grad():
        for n, (att, f) in enumerate(zip(atts, feats)):
            ref_l = torch.sigmoid(att.feat_att_left(f))
            ref_r = torch.sigmoid(att.feat_att_right(f.flip(-1)))
            ref_l64 = torch.sigmoid(att.feat_att_left.double()(f.double())).float()
            assert outs[2 * n].shape == ref_l.shape
            assert (outs[2 * n] - ref_l).abs().max().item() < 2e-5
            assert (outs[2 * n + 1] - ref_r).abs().max().item() < 2e-5
            assert (outs[2 * n] - ref_l64).abs().max().item() < 2e-5
            att.feat_att_left.float()


def test_feature_gates_deterministic_and_refuse_bad_jobs():
    att = _att(16, 3)
    f = torch.rand(4, 1, 68, 120, device="cuda")
    w = ops.feature_gate_weights(att.feat_att_left)
    a = ops.feature_gates([(f, w)])[0]
    b = ops.feature_gates([(f, w)])[0]
    assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        ops.feature_gates([(torch.rand(2, 2, 8, 8, device="cuda"), w)])
    with pytest.raises(RuntimeError):
        ops.feature_gates([(f, w)] * 9)
