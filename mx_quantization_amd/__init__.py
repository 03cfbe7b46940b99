"""mx_quantization_amd -- MI355X-native MX-quantized, approximator-pruned top-k attention.

The hot path of d9bjo0522/mx_quantization rebuilt for gfx950: hand-written HIP
kernels behind a C ABI (include/mxa.h, libmxa.so), driven from Python on
PyTorch-ROCm, exposed through

  * `mx_topk_attention` -- the fused path (MXINT8 QK^T, approximate scores,
    exact-order top-k, softmax, MXINT8 P.V),
  * `mx_qkv_attention` -- the qkv mx.Linear fused in front of it (x -> MX operands),
  * `mx_approx_scores` -- the approximator's scores alone (pred = aQ @ aK^T, ELSA),
  * `topk` -- torch.topk with torch's CPU index order (and the prune mask), on the device,
  * the reference's own operator surface, as drop-in packages:
      mx_quantization_amd.mx     (microxscaling `mx`: matmul, quantize_mx_op, ...)
      mx_quantization_amd.funcs  (`funcs`: exponent_approximation, ...)
    `install_dropin()` registers them as top-level `mx` / `funcs` so the
    patched attention modules import them unchanged.
"""
from ._native import NativeError, lib  # noqa: F401
from .ops import (  # noqa: F401
    approx_values,
    elsa_cos_table,
    mx_approx_scores,
    LinearWeightMX,
    mx_linear,
    mx_matmul,
    mx_qkv_attention,
    mx_topk_attention,
    mx_topk_attention_proj,
    quantize_bfloat,
    quantize_mx,
    shared_exponents,
    topk,
    unpack_mask,
)

from .exact_topk import TORCH as exact_topk_torch, bind_exact_topk, unbind_exact_topk  # noqa: F401,E402

__all__ = ["bind_exact_topk", "unbind_exact_topk", "exact_topk_torch", "mx_topk_attention", "mx_qkv_attention", "mx_topk_attention_proj", "mx_linear", "LinearWeightMX", "mx_approx_scores", "topk", "unpack_mask", "quantize_mx", "mx_matmul", "install_dropin", "NativeError"]


def install_dropin():
    """Make `import mx`, `from mx.mx_ops import ...`, `from funcs import ...`
    resolve to this package's drop-in surfaces."""
    import importlib
    import sys

    for top, pkg in (("mx", "mx_quantization_amd.mx"), ("funcs", "mx_quantization_amd.funcs")):
        mod = importlib.import_module(pkg)
        sys.modules[top] = mod
        for sub in getattr(mod, "_SUBMODULES", ()):
            sys.modules[f"{top}.{sub}"] = importlib.import_module(f"{pkg}.{sub}")
    return sys.modules["mx"], sys.modules["funcs"]
