"""CPU-offload wrapper with the reference's API (mapreduce_v2/cpu_offload_wrapper.py:14-83),
designed for an MI355X's 288 GB of HBM.

The reference exists to squeeze Booster-sized inference into a small GPU: the stereo
model (or the tiler around it) and the mono model are moved onto the device only while
they run (``temporarily_to``), the mono maps are parked on the host between the two
stages, and the allocator cache is emptied afterwards.  On an MI355X the whole working
set of a Booster tile (a few GB) is a small fraction of HBM, so the build
keeps weights and mono maps resident: every stage already on the target device is a
no-op move, exactly like the reference's own ``temporarily_to`` when devices match.
The observable behaviour is the reference's:

* same constructor ``CPUOffloadWrapper(model, mono_model=None, offload_feature=True,
  offload_mono=True)`` and forward ``(left, right, mono_left=None, mono_right=None,
  *args, **kwargs)``; extra arguments go to the wrapped model unchanged;
* without mono maps the mono model is called as ``mono_model(left, right)`` (line 67;
  the reference's call convention, not DAv2's), and without one either a ``ValueError``
  with the reference's message is raised;
* modules that live elsewhere (e.g. on the host) are moved to the input's device for
  their stage and moved back afterwards (``temporarily_to``);
* with ``offload_mono`` the mono maps make the host round trip only when
  ``host_roundtrip=True``: values are unchanged by it, so by default they stay in HBM;
* ``release_cache`` (default False) empties the caching allocator after the forward as the
  reference always does (line 82); on MI355X that only forces re-allocation next call.

The model computes fp32: ``mixed_precision`` reaches the wrapped model through ``kwargs``
as in the reference (where the tiler drops it) and autocast is not entered.
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import Iterator, Optional

import torch
import torch.nn as nn

Tensor = torch.Tensor


def _device_of(module: nn.Module) -> Optional[torch.device]:
    p = next(module.parameters(), None)
    return None if p is None else p.device


@contextmanager
def temporarily_to(module: nn.Module, device: torch.device) -> Iterator[nn.Module]:
    """cpu_offload_wrapper.py:14-26: move ``module`` to ``device`` for the block and back."""
    original = _device_of(module)
    moved = original is not None and original != torch.device(device)
    if moved:
        module.to(device)
    try:
        yield module
    finally:
        if moved:
            module.to(original)


class CPUOffloadWrapper(nn.Module):
    """cpu_offload_wrapper.py:28-83 (see the module docstring for the HBM-resident policy)."""

    def __init__(self, model: nn.Module, mono_model: Optional[nn.Module] = None, offload_feature: bool = True,
                 offload_mono: bool = True, *, host_roundtrip: bool = False, release_cache: bool = False) -> None:
        super().__init__()
        self.model = model
        self.mono_model = mono_model
        self.offload_feature = offload_feature
        self.offload_mono = offload_mono
        self.host_roundtrip = host_roundtrip
        self.release_cache = release_cache

    @staticmethod
    def _detach_to_cpu(tensor: Optional[Tensor]) -> Optional[Tensor]:
        return None if tensor is None else tensor.detach().to("cpu")

    def forward(self, left: Tensor, right: Tensor, mono_left: Optional[Tensor] = None,
                mono_right: Optional[Tensor] = None, *args, **kwargs):
        device = left.device
        if mono_left is None or mono_right is None:
            if self.mono_model is None:
                raise ValueError("Monocular model required when mono inputs absent")
            with temporarily_to(self.mono_model, device):
                mono_left, mono_right = self.mono_model(left, right)
            if self.offload_mono:
                if self.host_roundtrip:
                    mono_left, mono_right = self._detach_to_cpu(mono_left), self._detach_to_cpu(mono_right)
                else:
                    mono_left, mono_right = mono_left.detach(), mono_right.detach()
        with temporarily_to(self.model, device):
            if mono_left is not None and mono_left.device != device:
                mono_left = mono_left.to(device)
            if mono_right is not None and mono_right.device != device:
                mono_right = mono_right.to(device)
            disparity = self.model(left, right, mono_left, mono_right, *args, **kwargs)
        if self.release_cache and device.type == "cuda":
            torch.cuda.empty_cache()
        return disparity
