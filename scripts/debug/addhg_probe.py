"""n_additional_hourglass = 2 on the GPU model: each hourglass's output against the same module
run on the CPU from the captured GPU input."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from stereoanywhere_amd import synth  # noqa: E402
from stereoanywhere_amd.model import StereoAnywhere  # noqa: E402

m = StereoAnywhere(dict(n_additional_hourglass=2)).eval()
synth.load_seeded_weights(m, 0)
m = m.cuda()
cap = {}


def hook(name):
    def h(mod, inp, out):
        cap[name] = ([x.detach().cpu() if torch.is_tensor(x) else [f.detach().cpu() for f in x] for x in inp],
                     out.detach().cpu() if torch.is_tensor(out) else None)
    return h


m.hourglass_mono.register_forward_hook(hook("hg0"))
m.hourglass_mono_stack[1].register_forward_hook(hook("hg1"))
m.hourglass_mono_stack[2].register_forward_hook(hook("hg2"))
pb = synth.synthetic_batch(1, 128, 256, 48.0, seed0=3)
x = [torch.from_numpy(pb[k]).cuda() for k in ("left", "right", "mono_left", "mono_right")]
with torch.no_grad():
    m(*x, iters=1, test_mode=True)
print("captured", sorted(cap))
mc = StereoAnywhere(dict(n_additional_hourglass=2)).eval()
synth.load_seeded_weights(mc, 0)
for name, mod in (("hg0", mc.hourglass_mono), ("hg1", mc.hourglass_mono_stack[1]), ("hg2", mc.hourglass_mono_stack[2])):
    if name not in cap:
        continue
    inp, out = cap[name]
    with torch.no_grad():
        ref = mod(*inp)
    print(name, "in", tuple(inp[0].shape), "max|gpu-cpu|", float((out - ref).abs().max()), "max", float(ref.abs().max()))
