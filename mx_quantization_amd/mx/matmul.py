"""MX matmul -- drop-in for microxscaling/mx/matmul.py (forward / inference).

in1 is quantized along its last axis, in2 along its second-to-last, and the
product of the int8 codes runs on int8 MFMA with exact per-block epilogues
(libmxa.so: mxa_matmul)."""
from __future__ import annotations

import torch

from .. import ops
from .elemwise_ops import quantize_elemwise_op
from .formats import ElemFormat, INT_MBITS
from .specs import apply_mx_specs, mx_assert_test

torch_matmul = torch.matmul


def _mbits(fmt):
    if isinstance(fmt, str):
        fmt = ElemFormat.from_str(fmt)
    if fmt not in (ElemFormat.int8, ElemFormat.int4):
        raise NotImplementedError(f"mx.matmul element format {fmt}: int8 / int4 are built")
    return INT_MBITS[fmt]


def _check_specs(s):
    if s["block_size"] != 32 or (s["scale_bits"] not in (0, 8)) or s["shared_exp_method"] != "max":
        raise NotImplementedError("mx.matmul on the device needs block_size 32, scale_bits 8, 'max' exponents")
    if s["round_mx_output"] != "nearest":
        raise NotImplementedError("mx.matmul on the device rounds MX elements to nearest")


def matmul(in1, in2, bias=None, mx_specs=None, name=None, mode_config="aa"):
    """matmul.py:211-222 -> MatMulFunction.forward :31-100."""
    mx_assert_test(mx_specs)
    if mx_specs is None:
        return torch_matmul(in1, in2) if bias is None else torch.addmm(bias, in1, in2)
    s = apply_mx_specs(mx_specs)
    assert mode_config in ("aa", "aw", "wa")
    f1 = s["a_elem_format"] if mode_config[0] == "a" else s["w_elem_format"]
    f2 = s["a_elem_format"] if mode_config[1] == "a" else s["w_elem_format"]
    bf1 = quantize_elemwise_op(in1, mx_specs=s, round=s["round_output"])
    bf2 = quantize_elemwise_op(in2, mx_specs=s, round=s["round_output"])
    if f1 is None or f2 is None:
        raise NotImplementedError("mx.matmul with an unquantized operand")
    _check_specs(s)
    # each operand is quantized in its own dtype; torch_matmul returns the autocast dtype
    # under torch.autocast (P float16 @ V float32 in the autocast DeiT eval), else the
    # operands' common dtype (mismatched dtypes raise, as torch.matmul does)
    out = ops.mx_matmul(bf1, bf2, _mbits(f1), _mbits(f2), flush=s["mx_flush_fp32_subnorms"],
                        out_dtype=ops.autocast_dtype(bf1.device.type))
    out = quantize_elemwise_op(out, mx_specs=s, round=s["round_output"])
    if bias is not None:
        out = out + quantize_elemwise_op(bias, mx_specs=s, round=s["round_weight"])
        out = quantize_elemwise_op(out, mx_specs=s, round=s["round_output"])
    return out
