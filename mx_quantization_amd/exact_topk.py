"""torch.topk in torch's CPU index order for the UNCHANGED attention modules.

The patched modules call `torch.topk(pred_scores, self.k, dim=-1, largest=True,
sorted=True)` themselves (workloads/deit/scripts/main.py:123, :127,
workloads/DiT/models.py:194, :199, workloads/PixArt/models/MX_transformer_block.py:678,
:825).  On ROCm that is torch's GPU top-k, whose order among tied scores differs from
the CPU path the reference's results come from.  Rather than patch
torch for the whole process, `bind_exact_topk(module)` rebinds the name `torch` inside
the given modules to `TORCH`: a namespace that forwards every attribute to torch except
`topk`, which runs mxa_topk (include/mxa.h) on device tensors:

    import mx_quantization_amd as M
    M.install_dropin()
    import models                      # the workload module (deit main.py, DiT models.py)
    M.bind_exact_topk(models)          # its `torch.topk(...)` calls now give CPU order

Covered: device tensors of float32 / float16 / bfloat16, the last dim, largest=True,
sorted=True (the only form the modules use), up to 1,024 columns (include/mxa.h
kWMaxN: the PixArt 512x512 self-attention rows; longer rows raise NativeError,
MXA_ERR_UNSUPPORTED).  Other forms (largest=False,
sorted=False, another dim, CPU tensors) are torch's own topk, unchanged.
"""
from __future__ import annotations

import types

import torch

from . import ops


def topk(input, k, dim=-1, largest=True, sorted=True, *, out=None):
    """torch.topk with torch's CPU index order on device tensors (TopKImpl.h:45-86)."""
    last = dim == -1 or (input.dim() > 0 and dim == input.dim() - 1)
    if (out is None and last and largest and sorted and input.is_cuda and input.dim() > 0
            and input.dtype in (torch.float32, torch.float16, torch.bfloat16)):
        if not 0 <= k <= input.shape[-1]:
            raise RuntimeError(f"selected index k out of range (k={k}, n={input.shape[-1]})")
        vals, idx = ops.topk(input, int(k))
        return torch.return_types.topk((vals, idx))
    if out is not None:
        return torch.topk(input, k, dim=dim, largest=largest, sorted=sorted, out=out)
    return torch.topk(input, k, dim=dim, largest=largest, sorted=sorted)


class _TorchNamespace(types.ModuleType):
    """`torch` for a rebound module: every attribute is torch's, except topk."""

    def __init__(self):
        super().__init__("torch", "torch with topk in CPU index order (mx_quantization_amd.exact_topk)")
        self.topk = topk

    def __getattr__(self, name):
        return getattr(torch, name)

    def __dir__(self):
        return sorted(set(dir(torch)) | {"topk"})


TORCH = _TorchNamespace()


def bind_exact_topk(*modules):
    """Rebind `torch` to TORCH in each module (a module object or its globals dict) whose
    global `torch` is the torch package; returns the number of modules rebound."""
    n = 0
    for m in modules:
        g = m if isinstance(m, dict) else vars(m)
        if g.get("torch") is torch:
            g["torch"] = TORCH
            n += 1
    return n


def unbind_exact_topk(*modules):
    """Undo bind_exact_topk."""
    for m in modules:
        g = m if isinstance(m, dict) else vars(m)
        if g.get("torch") is TORCH:
            g["torch"] = torch
