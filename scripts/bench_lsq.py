"""Time sa_weighted_lsq alone at the model's size (B samples x 136*240)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from stereoanywhere_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2 * 136 * 240  # both maps of a pair
for (B, spread), single in [(c, sb) for c in ((1, 1.0), (4, 1.0), (64, 1.0), (4, 0.01), (4, 0.0))
                            for sb in (False, True)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    m = torch.rand(B, n, device="cuda", generator=g)
    # spread 0.01: clustered disparities (few bins per wave in the low digits); 0: all equal
    d = (40 * m + 3) * spread + 5 + torch.randn(B, n, device="cuda", generator=g) * spread
    c = torch.rand(B, n, device="cuda", generator=g)
    for _ in range(3):
        ops.weighted_lsq(m, d, c, single_block=single)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.weighted_lsq(m, d, c, single_block=single)
    e1.record()
    torch.cuda.synchronize()
    print(f"B={B} n={n} spread={spread} single_block={single}: {e0.elapsed_time(e1) / 20 * 1000:.1f} us")
