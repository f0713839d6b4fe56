"""GPU (MIOpen) vs CPU torch of the unfused hourglass chain (n_additional_hourglass = 2) on a
one-hot masked volume: how far the classifier output moves between the two backends."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

torch.backends.cudnn.benchmark = False
for nadd in (0, 2):
    m = StereoAnywhere(dict(n_additional_hourglass=nadd)).eval()
    synth.load_seeded_weights(m, 0)
    g = torch.Generator().manual_seed(0)
    B, H, W1, W2 = 1, 32, 64, 64
    v = torch.randn(B, 1, W2, H, W1, generator=g)
    bins = torch.randint(0, 8, (B, 1, 1, H, W1), generator=g)
    binr = torch.randint(0, 8, (B, 1, W2, H, 1), generator=g)
    n = torch.arange(8).view(1, 8, 1, 1, 1)
    x = v * ((bins == n) & (binr == n)).float()
    mm = torch.rand(B, 1, 128, 256, generator=g)
    fl = [F.interpolate(mm, scale_factor=1 / 2 ** i, mode="bilinear", align_corners=True) for i in range(2, 6)]
    cls = m.classifier_mono.weight.permute(0, 1, 4, 2, 3).contiguous()
    outs = []
    for dev in ("cpu", "cuda"):
        mm_ = m.to(dev)
        with torch.no_grad():
            a = mm_.hourglass_mono(x.to(dev), [f.to(dev) for f in fl], [f.to(dev) for f in fl])
            for i in range(nadd):
                hg = mm_.hourglass_mono_stack[i]
                a = hg(a, [f.to(dev) for f in fl], [f.to(dev) for f in fl])
            outs.append(F.conv3d(a, cls.to(dev), padding=1).cpu())
    d = (outs[0] - outs[1]).abs()
    print(f"n_additional={nadd}: max|cpu-gpu| {float(d.max()):.3e} of max {float(outs[0].abs().max()):.3e}; "
          f"softmax-disp max diff {float((torch.softmax(outs[0], 2) - torch.softmax(outs[1], 2)).abs().max()):.3e}",
          flush=True)
    with torch.no_grad():
        xc = x.cuda()
        c1 = F.conv3d(xc, m.hourglass_mono.down_layers[0][0].conv.weight.cuda() if hasattr(m.hourglass_mono.down_layers[0][0], "conv") else None, stride=2, padding=1) if False else None
