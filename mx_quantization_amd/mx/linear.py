"""MX Linear -- drop-in for microxscaling/mx/linear.py (forward / inference).

out = MX(x, along in_features) @ MX(W, along in_features)^T (+ bias), on the
device: float32 inputs through mxa_linear (the block-scaled int8-MFMA GEMM with the
weight prepared once per weight version), other dtypes through mxa_matmul.  This is the
qkv / proj projection around the attention core (a SURVEY §8f "next" row) as the
patched modules' `from mx import Linear` sees it.  The fused forms are
mx_quantization_amd.mx_qkv_attention (qkv Linear -> attention operands, and with
proj_weight the proj Linear behind it: include/mxa.h mxa_attention_proj)."""
from __future__ import annotations

import torch

from .. import ops
from .elemwise_ops import quantize_elemwise_op
from .matmul import _check_specs, _mbits
from .specs import apply_mx_specs, mx_assert_test


# id(weight) -> (weakref to the weight, stamp, LinearWeightMX).  The entry belongs to
# the weight OBJECT (the weakref must still resolve to it), so a new tensor that the
# caching allocator puts at a freed weight's address never sees the old codes, and an
# entry dies with its weight (weakref callback).  The stamp adds what can change in
# place: storage address, shape, strides, device, the autograd version counter and the
# specs.  In-place writes that bypass the version counter (`param.data.copy_(...)`) are
# invisible to it: call invalidate_prepared() after them.
_PREPARED = {}


def invalidate_prepared(weight=None):
    """Drop the prepared MX codes of `weight` (all weights when None)."""
    if weight is None:
        _PREPARED.clear()
    else:
        _PREPARED.pop(id(weight), None)


def _prepared_weight(weight, s):
    """The weight's MX codes, prepared once per weight version (inference: constant)."""
    import weakref
    stamp = (weight.data_ptr(), tuple(weight.shape), tuple(weight.stride()), str(weight.device), weight._version,
             bool(s["mx_flush_fp32_subnorms"]), int(s["bfloat"]))
    ent = _PREPARED.get(id(weight))
    if ent is not None and ent[0]() is weight and ent[1] == stamp:
        return ent[2]
    wq = ops.LinearWeightMX(weight.detach().contiguous(), weight.shape[0], s["mx_flush_fp32_subnorms"], s["bfloat"])
    wid = id(weight)
    ref = weakref.ref(weight, lambda _r, wid=wid: _PREPARED.pop(wid, None) if _PREPARED.get(wid, (None,))[0] is _r
                      else None)
    _PREPARED[wid] = (ref, stamp, wq)
    return wq


def linear(input, weight, bias=None, mx_specs=None, prequantized_weights=False, name=None):
    """LinearFunction.forward (linear.py:20-103)."""
    if mx_specs is None:
        return torch.nn.functional.linear(input, weight, bias)
    s = apply_mx_specs(mx_specs)
    _check_specs(s)
    if (input.dtype == torch.float32 and weight.dtype == torch.float32 and not prequantized_weights
            and _mbits(s["a_elem_format"]) == 8 and _mbits(s["w_elem_format"]) == 8
            and (bias is None or bias.dtype == torch.float32)
            and all(s.get(r, "nearest") == "nearest" for r in ("round_output", "round_weight", "round_mx_output"))):
        # mxa_linear: bf(x), MX along in_features, exact-then-rounded product, bf(out + bf(bias))
        wq = _prepared_weight(weight, s)
        return ops.mx_linear(input, wq, bias, flush_subnormals=s["mx_flush_fp32_subnorms"], bfloat=s["bfloat"],
                             autocast=ops.autocast_dtype(input.device.type))
    bf_in = quantize_elemwise_op(input, mx_specs=s, round=s["round_output"])
    bf_w = weight if prequantized_weights else quantize_elemwise_op(weight, mx_specs=s, round=s["round_weight"])
    x2 = bf_in.reshape(1, -1, bf_in.shape[-1])
    # f_linear under torch.autocast returns the autocast dtype (then + the fp32 bias
    # promotes to fp32, linear.py:88-101); outside it the operands' dtypes must agree
    out = ops.mx_matmul(x2, bf_w.t().unsqueeze(0), _mbits(s["a_elem_format"]), _mbits(s["w_elem_format"]),
                        flush=s["mx_flush_fp32_subnorms"], out_dtype=ops.autocast_dtype(x2.device.type))
    out = out.reshape(bf_in.shape[:-1] + (weight.shape[0],))
    out = quantize_elemwise_op(out, mx_specs=s, round=s["round_output"])
    if bias is not None:
        bb = bias if prequantized_weights else quantize_elemwise_op(bias, mx_specs=s, round=s["round_weight"])
        out = quantize_elemwise_op(out + bb, mx_specs=s, round=s["round_output"])
    return out


class Linear(torch.nn.Linear):
    """linear.py:227-320 (inference)."""

    def __init__(self, in_features, out_features, bias=True, mx_specs=None, name=None):
        mx_assert_test(mx_specs)
        self.mx_none = mx_specs is None
        self.name = name
        self.prequantized_weights = False
        self.mx_specs = apply_mx_specs(mx_specs)
        super().__init__(in_features, out_features, bias)

    def apply_mx_specs(self, mx_specs):
        mx_assert_test(mx_specs)
        self.mx_none = mx_specs is None
        self.mx_specs = apply_mx_specs(mx_specs)

    def append_name(self, postfix):
        self.name += postfix

    def get_quantized_weight(self):
        """The MX-quantized weight (linear.py:253-274)."""
        if self.mx_none:
            return self.weight
        from .mx_ops import quantize_mx_op
        bf_w = quantize_elemwise_op(self.weight, mx_specs=self.mx_specs, round=self.mx_specs["round_weight"])
        return quantize_mx_op(bf_w, self.mx_specs, elem_format=self.mx_specs["w_elem_format"], axes=[-1],
                              round=self.mx_specs["round_mx_output"])

    def forward(self, inputs):
        if self.mx_none:
            return super().forward(inputs)
        return linear(inputs, self.weight, self.bias, self.mx_specs, self.prequantized_weights, self.name)
