"""MX quantization ops -- drop-in for microxscaling/mx/mx_ops.py.

Arithmetic runs in libmxa.so on the MI355X (mxa_quantize_mx, mxa_shared_exponents).
_reshape_to_blocks / _undo_reshape_to_blocks are view/pad plumbing with the
reference's exact shape semantics (mx_ops.py:102-174).

Scope: integer element formats (int8 / int4 / int2), one shared axis, shared
exponent method "max" -- everything the attention path and its callers use.
Float element formats (fp8/fp6/fp4) raise NotImplementedError.
"""
from __future__ import annotations

import torch

from .. import ops
from .formats import ElemFormat, INT_MBITS, RoundingMode  # noqa: F401
from .specs import mx_assert_test


def _shared_exponents(A, method="max", axes=None, ebits=0):
    """floor(log2(max|A| over axes)) with the 2^-126 zero trick and the optional
    [-emax, emax] clamp (mx_ops.py:49-99).  method "none" is elementwise."""
    if method not in ("max", "none"):
        raise Exception("Unrecognized shared exponent selection method %s" % method)
    if method == "none":
        return ops.shared_exponents(A, "none", ebits=ebits)
    if axes is None:
        return ops.shared_exponents(A.reshape(1, -1), "max", axis=-1, block_size=0, ebits=ebits).reshape(())
    axes = [a % A.dim() for a in axes]
    if len(axes) > 1:
        # max is exact and order-free: fold the other axes first, keep them as size 1
        A = torch.amax(A.abs(), dim=axes[1:], keepdim=True)
    return ops.shared_exponents(A, "max", axis=axes[0], block_size=0, ebits=ebits)


def _reshape_to_blocks(A, axes, block_size):
    """Tile axis -> (nblocks, block_size) with zero padding (mx_ops.py:102-161)."""
    if axes is None:
        raise Exception("axes required in order to determine which dimension toapply block size to")
    if block_size == 0:
        raise Exception("block_size == 0 in _reshape_to_blocks")
    axes = sorted(x + A.dim() if x < 0 else x for x in axes)
    for i in range(len(axes)):
        axes[i] += i
        A = torch.unsqueeze(A, dim=axes[i] + 1)
    orig_shape = A.size()
    pad = [0, 0] * len(orig_shape)
    do_padding = False
    for axis in axes:
        L = orig_shape[axis]
        if L % block_size:
            pad[2 * axis] = block_size - L % block_size
            do_padding = True
    if do_padding:
        A = torch.nn.functional.pad(A, list(reversed(pad)), mode="constant")
    padded_shape = A.size()
    shape = list(padded_shape)
    for axis in axes:
        if shape[axis] >= block_size:
            assert shape[axis] % block_size == 0
            shape[axis + 1] = block_size
            shape[axis] = shape[axis] // block_size
        else:
            shape[axis + 1] = shape[axis]
            shape[axis] = 1
    return A.view(shape), axes, orig_shape, padded_shape


def _undo_reshape_to_blocks(A, padded_shape, orig_shape, axes):
    """Inverse of _reshape_to_blocks (mx_ops.py:164-174)."""
    A = A.view(padded_shape)
    if list(padded_shape) != list(orig_shape):
        A = A[tuple(slice(0, x) for x in orig_shape)]
    for axis in reversed(axes):
        A = torch.squeeze(A, dim=axis + 1)
    return A


def _quantize_mx(A, scale_bits, elem_format, shared_exp_method="max", axes=None, block_size=0,
                 round="nearest", flush_fp32_subnorms=False, custom_cuda=False, predict_phase=False,
                 bfloat=0):
    """MX quantize (mx_ops.py:180-306) on the device.  custom_cuda is accepted and
    ignored: there is one implementation, the HIP kernel."""
    if elem_format is None:
        return A
    if isinstance(elem_format, str):
        elem_format = ElemFormat.from_str(elem_format)
    if elem_format not in INT_MBITS:
        raise NotImplementedError(f"MX element format {elem_format.name}: only int8/int4/int2 are built")
    if shared_exp_method != "max":
        raise NotImplementedError("shared_exp_method must be 'max'")
    if predict_phase:
        raise NotImplementedError("predict_phase epsilon hack (elemwise_ops.py:79-85) is not built")
    assert scale_bits > 0
    axes = [axes] if isinstance(axes, int) else list(axes)
    if len(axes) != 1:
        raise NotImplementedError("MX quantization over more than one axis")
    return ops.quantize_mx(A, elem_mbits=INT_MBITS[elem_format], block_size=block_size, axis=axes[0],
                           scale_bits=scale_bits, round=round, flush=flush_fp32_subnorms, bfloat=bfloat)


def quantize_mx_op(A, mx_specs: dict, elem_format=None, block_size=None, axes=None, round="nearest",
                   expand_and_reshape=False, predict_phase=False):
    """Spec-level MX quantize (mx_ops.py:309-341)."""
    mx_assert_test(mx_specs)
    if elem_format is None:
        return A
    if isinstance(elem_format, str):
        elem_format = ElemFormat.from_str(elem_format)
    if block_size is None:
        block_size = mx_specs["block_size"]
    scale_bits = 8 if mx_specs["scale_bits"] == 0 else mx_specs["scale_bits"]
    return _quantize_mx(A, scale_bits, elem_format, block_size=block_size, axes=axes, round=round,
                        shared_exp_method=mx_specs["shared_exp_method"],
                        flush_fp32_subnorms=mx_specs["mx_flush_fp32_subnorms"],
                        custom_cuda=mx_specs["custom_cuda"], predict_phase=predict_phase)
