"""Load reference checkpoints (test.py:140-152: DataParallel 'module.' prefix, optional
'state_dict' wrapper, strict=True) into the MI355X model.  Only tensors are read:
``torch.load(..., weights_only=True)``."""
from __future__ import annotations

import torch


def strip_module_prefix(sd):
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in sd.items()}


def load_reference_checkpoint(model: torch.nn.Module, ckpt, strict: bool = True):
    if isinstance(ckpt, str):
        ckpt = torch.load(ckpt, map_location="cpu", weights_only=True)
    sd = ckpt["state_dict"] if isinstance(ckpt, dict) and "state_dict" in ckpt else ckpt
    return model.load_state_dict(strip_module_prefix(sd), strict=strict)
