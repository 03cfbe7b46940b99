"""mx_specs configuration -- the reference's config surface
(microxscaling/mx/specs.py:61-363): same keys, defaults, merge rules and errors.
Pure configuration plumbing; no arithmetic lives here."""
from __future__ import annotations

import argparse
import collections
import json
import os
import traceback

_ASSERT_MODE = os.environ.get("MX_ASSERT", "False")

# key -> (default, help).  Defaults as specs.py:81-120.
_SPEC_TABLE = {
    "scale_bits": (0, "Bits (sign + magnitude) to use for shared exponent/scale"),
    "w_elem_format": (None, "Weight MX elem format, one of {fp8_e5m2, fp8_e4m3, fp6_e3m2, fp6_e2m3, fp4_e2m1, int8, int4}"),
    "a_elem_format": (None, "Activation MX elem format. See w_elem_format"),
    "w_elem_format_bp": (None, "Backpass weight MX elem format. See w_elem_format"),
    "a_elem_format_bp": (None, "Backpass stashed activation MX elem format. See w_elem_format"),
    "a_elem_format_bp_ex": (None, "Backpass act (grad) MX elem format. See w_elem_format"),
    "a_elem_format_bp_os": (None, "Backpass act (grad) MX elem format. See w_elem_format"),
    "mx_flush_fp32_subnorms": (False, "MX quantization flushes blocks with subnormal shared scale to zero"),
    "shared_exp_method": ("max", "Shared exponent calculation method. Options: max, none"),
    "block_size": (0, "mx shared exponent block size"),
    "bfloat": (0, "BfloatX format (8exp + sign + mantissa). Only one of bfloat or fp can be used"),
    "fp": (0, "fpX format (5exp + sign + mantissa). Only one of bfloat or fp can be used"),
    "bfloat_subnorms": (True, "Bfloat/FP supports subnorms"),
    "quantize_backprop": (True, "Enable mx/bfloat quantization on backward pass"),
    "round": ("nearest", "Global rounding mode. Choices: nearest, floor"),
    "round_m": ("nearest", "ADAM optimizer m and v rounding mode"),
    "round_weight": ("nearest", "Weight bfloat rounding mode (W in WAGE)"),
    "round_output": ("nearest", "Activation bfloat rounding mode (A in WAGE)"),
    "round_grad_weight": ("nearest", "Weight update rounding mode (G in WAGE)"),
    "round_grad_input": ("nearest", "Error gradient rounding mode (E in WAGE)"),
    "round_mx_output": ("nearest", "Forward pass mx rounding mode"),
    "round_mx_input_grad_input": ("nearest", ""),
    "round_mx_weight_grad_input": ("nearest", ""),
    "round_mx_grad_output_grad_input": ("nearest", ""),
    "round_mx_input_grad_weight": ("nearest", ""),
    "round_mx_grad_output_grad_weight": ("nearest", ""),
    "softmax_exp2": (False, "Softmax uses 2^x instead of e^x"),
    "vec_use_exp2": (False, "Use 2^x to compute e^x"),
    "vec_use_recip": (False, "Use 1/x to compute division"),
    "custom_cuda": (False, "Enable custom CUDA kernels for quantization"),
}


class MxSpecs(collections.UserDict):
    """dict of MX options with the reference's defaults (specs.py:61-181)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.help_strings = {k: h for k, (_, h) in _SPEC_TABLE.items()}
        for k, (default, _) in _SPEC_TABLE.items():
            if k not in self.data:
                self.data[k] = default
        for k in self.data:
            assert k in self.help_strings, f"Unknown key '{k}' in mx specs"

    def safe_json(self, indent=None):
        return json.dumps(self.data, indent=indent,
                          default=lambda o: f"<<non-serializable: {type(o).__qualname__}>>")

    def __str__(self):
        return self.safe_json(indent=4)


def get_default_mx_specs():
    return MxSpecs()


def get_backwards_mx_specs(specs):
    """A no-quantize spec for backward when quantize_backprop is False (specs.py:136-156)."""
    bspecs = specs.copy()
    if not bspecs["quantize_backprop"]:
        for k in ("w_elem_format", "a_elem_format", "w_elem_format_bp", "a_elem_format_bp",
                  "a_elem_format_bp_os", "a_elem_format_bp_ex"):
            bspecs[k] = None
        bspecs["block_size"] = 0
        bspecs["bfloat"] = 0
        bspecs["fp"] = 0
    return bspecs


def apply_mx_specs(mx_specs, default_mx_specs=None):
    """Overlay the non-None entries of mx_specs on the defaults (specs.py:159-178)."""
    if not default_mx_specs:
        default_mx_specs = get_default_mx_specs()
    if not mx_specs:
        return default_mx_specs
    for k in mx_specs:
        if mx_specs[k] is not None:
            if k not in default_mx_specs:
                raise KeyError(f"Unknown key '{k}' passed to mx specs")
            default_mx_specs[k] = mx_specs[k]
    return default_mx_specs


def add_mx_args(parser: argparse.ArgumentParser) -> argparse.ArgumentParser:
    """CLI flags for every spec, typed from its default (specs.py:181-224)."""
    group = parser.add_argument_group("mx", "MX specs")
    group.add_argument("--mx_dir", type=str, default=None, help="Path to mx library")
    for k, (v, h) in _SPEC_TABLE.items():
        h = h or "No help string"
        if "elem_format" in k:
            group.add_argument("--" + k, type=str, default=v, help=h)
        elif isinstance(v, bool) and v is False:
            group.add_argument("--" + k, action="store_true", help=h)
        elif isinstance(v, bool) and v is True:
            group.add_argument("--no_" + k, action="store_true", help=h)
        else:
            group.add_argument("--" + k, type=type(v), default=None, help=h)
    group.add_argument("--skip_early_exit", action="store_true", default=False,
                       help="Don't early exit if no quantization is specified")
    return parser


def finalize_mx_specs(specs, early_exit=True):
    """Resolve dependent specs (specs.py:227-274); None when nothing quantizes."""
    if (not specs.get("w_elem_format", 0) and not specs.get("a_elem_format", 0)
            and not specs.get("w_elem_format_bp", 0) and not specs.get("a_elem_format_bp", 0)
            and not specs.get("a_elem_format_bp_os", 0) and not specs.get("a_elem_format_bp_ex", 0)
            and not specs.get("bfloat", 0) and not specs.get("fp", 0) and early_exit):
        return None
    if specs.get("custom_cuda"):
        import torch
        assert torch.cuda.is_available(), "'custom_cuda' is only supported on CUDA devices."

    def fill(dst, src):
        if (dst not in specs or specs[dst] is None) and src in specs:
            specs[dst] = specs[src]

    for dst, src in (("w_elem_format_bp", "w_elem_format"), ("a_elem_format_bp", "a_elem_format"),
                     ("a_elem_format_bp_os", "a_elem_format"), ("a_elem_format_bp_ex", "a_elem_format"),
                     ("round_m", "round"), ("round_output", "round"), ("round_grad_weight", "round"),
                     ("round_grad_input", "round"), ("round_weight", "round"), ("round_mx_output", "round"),
                     ("round_mx_input_grad_input", "round_grad_input"),
                     ("round_mx_weight_grad_input", "round_grad_input"),
                     ("round_mx_grad_output_grad_input", "round_grad_input"),
                     ("round_mx_input_grad_weight", "round_grad_input"),
                     ("round_mx_grad_output_grad_weight", "round_grad_input")):
        fill(dst, src)
    return apply_mx_specs(specs, get_default_mx_specs())


def get_mx_specs(parsed_args: argparse.Namespace):
    """Specs from parsed CLI args (specs.py:277-299)."""
    parsed = {}
    for k, (v, _) in _SPEC_TABLE.items():
        if isinstance(v, bool) and v is True:
            if hasattr(parsed_args, "no_" + k):
                parsed[k] = not getattr(parsed_args, "no_" + k)
        elif hasattr(parsed_args, k):
            parsed[k] = getattr(parsed_args, k)
    early_exit = not getattr(parsed_args, "skip_early_exit", False)
    return finalize_mx_specs(parsed, early_exit=early_exit)


def mx_assert_test(mx_specs):
    """MX_ASSERT=True makes a None mx_specs an error (specs.py:351-363)."""
    if _ASSERT_MODE == "True" and mx_specs is None:
        stack = traceback.extract_stack()
        f1, f2 = stack[-2], stack[-3]
        raise ValueError("MX assert test failed!\n" + f"mx_specs is None in function {f1.name}\n"
                         + f"Called from {f2.filename}, line {f2.lineno}\n" + f"  {f2.line}")
