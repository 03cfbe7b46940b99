"""Elementwise quantization -- drop-in for microxscaling/mx/elemwise_ops.py.
bfloatX rounding runs in libmxa.so (mxa_quantize_bfloat)."""
from __future__ import annotations

import torch

from .. import ops


def _quantize_bfloat(A, bfloat, round="nearest", custom_cuda=False, allow_denorm=True):
    """bfloatX (8 exponent bits) quantization (elemwise_ops.py:201-216)."""
    if bfloat == 0 or bfloat == 32:
        return A
    return ops.quantize_bfloat(A, bfloat=bfloat, round=round, allow_denorm=allow_denorm)


def quantize_elemwise_op(A, mx_specs, round=None):
    """Spec-level elementwise quantization (elemwise_ops.py:243-277)."""
    if mx_specs is None:
        return A
    if round is None:
        round = mx_specs["round"]
    if (mx_specs["bfloat"] == 16 and round == "even" and torch.cuda.is_bf16_supported()
            and mx_specs["bfloat_subnorms"]):
        return A.to(torch.bfloat16)
    if mx_specs["bfloat"] > 0 and mx_specs["fp"] > 0:
        raise ValueError("Cannot set both [bfloat] and [fp] in mx_specs.")
    if mx_specs["bfloat"] > 9:
        return _quantize_bfloat(A, bfloat=mx_specs["bfloat"], round=round,
                                allow_denorm=mx_specs["bfloat_subnorms"])
    if 0 < mx_specs["bfloat"] <= 9:
        raise ValueError("Cannot set [bfloat] <= 9 in mx_specs.")
    if mx_specs["fp"] > 6:
        raise NotImplementedError("fpX elementwise formats are outside this build's scope")
    if 0 < mx_specs["fp"] <= 6:
        raise ValueError("Cannot set [fp] <= 6 in mx_specs.")
    return A
